#!/usr/bin/env python3
"""Launch durations of a single-stream run from a rocprofv3 kernel trace, for the
roofline's launch-time evidence (bench.py isolated_sample).

usage: isolated_sample.py <run_kernel_trace.csv> <out.csv> [--last N] [--min-us U] [--prefix P]
                          [--frames-per-launch B] [--prefix P]

Keeps, for every kernel named P... (default "void vip::": the library's) whose launches took
at least U us (default 5), its last N launches (default 300: the timed region and what
follows it, after bench.py's clock settle) that overlap no other launch. Writes one row per
launch: kernel (exact template signature, as vip_launched_kernels names it), index (its
position among that kernel's launches), duration_ns, frames_per_launch (B for a multi-frame
`..._frames_kernel<` of a `bench.py --batch B` run, else 1). The trace's argument list is cut off the
name, which then reads as vip_launched_kernels and the PMC summaries name the kernel.
Prints a per-kernel summary."""
import csv
import statistics
import sys


def strip_args(name: str) -> str:
    """'void vip::k<7, 16>(vip::StencilArgs)' -> 'void vip::k<7, 16>'"""
    return name[:name.rfind("(")] if name.endswith(")") else name


def main():
    args = sys.argv[1:]
    last = int(args[args.index("--last") + 1]) if "--last" in args else 300
    min_us = float(args[args.index("--min-us") + 1]) if "--min-us" in args else 5.0
    prefix = args[args.index("--prefix") + 1] if "--prefix" in args else "void vip::"
    fpl = int(args[args.index("--frames-per-launch") + 1]) if "--frames-per-launch" in args else 1
    rows = list(csv.DictReader(open(args[0])))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), strip_args(r["Kernel_Name"])) for r in rows)
    per = {}
    end_max = -1
    for i, (s, e, n) in enumerate(iv):
        nxt = iv[i + 1][0] if i + 1 < len(iv) else e
        tol = min(1000, (e - s) // 10)  # back-to-back launches touch by a few hundred ns in the trace
        alone = s >= end_max - tol and e <= nxt + tol
        end_max = max(end_max, e)
        per.setdefault(n, []).append((e - s, alone))
    with open(args[1], "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "index", "duration_ns", "frames_per_launch"])
        for n, ds in per.items():
            if not n.startswith(prefix) or statistics.median(d for d, _ in ds) < min_us * 1e3:
                continue
            keep = [(i, d) for i, (d, ok) in enumerate(ds) if ok][-last:]
            for i, d in keep:
                w.writerow([n, i, d, fpl if "_frames_kernel<" in n else 1])
            v = [d for _, d in keep]
            print(f"{len(v):5d} of {len(ds):6d} launches, mean {sum(v) / len(v) / 1e3:9.2f} us, median "
                  f"{statistics.median(v) / 1e3:9.2f} us: {n[:110]}")


if __name__ == "__main__":
    main()
