"""Summarise rocprofv3 --pmc passes (scripts/gpu_pmc.sh) into profiles/<tag>_pmc.json.

usage: python scripts/pmc_summary.py gpurun_out/pmc_c2 profiles/r01_c2_pmc.json [--frames-per-launch B]
Per kernel: mean of every counter over its dispatches. A multi-frame kernel
(`..._frames_kernel<`, bench.py --batch B) carries B frames per dispatch: its entry records
`frames_per_launch` so that bench.py divides its counts per frame. HBM traffic per launch
follows MI355X_MICROARCH.md's rocprofv3 section: FETCH_SIZE (KiB) counts 128-B
memory-side read requests at 64 B on gfx950, so it is doubled; WRITE_SIZE (KiB)
is taken as is. Both include Infinity-Cache hits (bench.py rotates 12 slabs,
> 256 MiB, so a frame's reads are mostly misses).
"""
import collections
import csv
import glob
import json
import os
import sys


def main(src, dst, fpl=1):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(src, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not name.startswith("void vip::"):
                continue
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"source": src, "kernels": {}}
    for name, ctrs in agg.items():
        means = {c: sum(v) / len(v) for c, v in ctrs.items()}
        k = {"dispatches": max(len(v) for v in ctrs.values()), "counters": means}
        if "FETCH_SIZE" in means and "WRITE_SIZE" in means:
            k["fetch_bytes_raw"] = means["FETCH_SIZE"] * 1024
            k["fetch_bytes"] = 2 * means["FETCH_SIZE"] * 1024
            k["write_bytes"] = means["WRITE_SIZE"] * 1024
            k["traffic_bytes"] = k["fetch_bytes"] + k["write_bytes"]
        if "_frames_kernel<" in name and fpl > 1:
            k["frames_per_launch"] = fpl
        out["kernels"][name.split("(")[0]] = k
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    for n, k in out["kernels"].items():
        print(n, {x: round(k[x] / 1e6, 2) for x in ("fetch_bytes", "write_bytes", "traffic_bytes") if x in k},
              {c: round(v) for c, v in k["counters"].items()})


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], int(a[a.index("--frames-per-launch") + 1]) if "--frames-per-launch" in a else 1)
