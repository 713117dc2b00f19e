"""Condense texture_ksize_bench.py output (stdin): one line per (build, k) with the guide-stage
and JBF kernel-stamped microseconds and the build's parity on a ragged frame."""
import json
import sys

for line in sys.stdin:
    if line.startswith("=="):
        print(line.strip())
        continue
    try:
        d = json.loads(line)
    except ValueError:
        continue
    u = d["us_per_launch"]
    g = [v for k, v in u.items() if "guide" in k][0]
    j = [v for k, v in u.items() if "guide" not in k][0]
    print(f"k{d['k']} guide {g:.1f} jbf {j:.1f} parity {d['parity']}")
