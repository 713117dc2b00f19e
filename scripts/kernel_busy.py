#!/usr/bin/env python3
"""Per-kernel launch durations and device busy time from a rocprofv3 kernel trace.

usage: kernel_busy.py <run_kernel_trace.csv> [out.json]

With frames in flight on several streams (bench.py --streams) launches overlap, so
the mean launch duration (what --stats averages) and the device time per launch
differ. This reports, per kernel name: launches, mean duration, the mean duration
of the launches that overlapped no other launch (the single-stream phase of
bench.py, which its roofline's avg_launch_ms times), and for the whole trace the
union of the launch intervals (device busy time) per launch."""
import csv
import json
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # launches that overlap no other launch
    # (sorted by start: a launch overlaps an earlier one iff it starts before their
    # latest end, a later one iff it ends after the next start). Back-to-back launches on
    # one stream can touch by a few hundred ns in the trace (the next start is stamped
    # before the previous end is; measured <= 156 ns), so an overlap below 1 us and below
    # a tenth of the launch does not count.
    iso = []
    end_max = -1
    for i, (s, e, _) in enumerate(iv):
        nxt = iv[i + 1][0] if i + 1 < len(iv) else e
        tol = min(1000, (e - s) // 10)
        iso.append(s >= end_max - tol and e <= nxt + tol)
        end_max = max(end_max, e)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    per = {}
    for (s, e, n), ok in zip(iv, iso):
        d = per.setdefault(n, {"launches": 0, "sum_ns": 0, "isolated": 0, "isolated_sum_ns": 0})
        d["launches"] += 1
        d["sum_ns"] += e - s
        if ok:
            d["isolated"] += 1
            d["isolated_sum_ns"] += e - s
    out = {"launches": len(iv), "busy_ns_per_launch": busy / max(1, len(iv)), "kernels": {}}
    for n, d in sorted(per.items(), key=lambda kv: -kv[1]["sum_ns"]):
        out["kernels"][n] = {"launches": d["launches"], "mean_us": round(d["sum_ns"] / d["launches"] / 1e3, 2),
                             "isolated_launches": d["isolated"],
                             "isolated_mean_us": round(d["isolated_sum_ns"] / d["isolated"] / 1e3, 2) if d["isolated"] else None}
    text = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
