#!/bin/bash
# Guide-stage tiles for R > 2 (round 6): texture_ksize_bench.py on each variant library,
# interleaved twice; run as gpu.sh py=... is not possible (a shell script), so:
#   gpurun -- 'bash scripts/experiments/run_gfb_ab.sh gfr_base gfr_A ... > gpurun_out/x.txt'
set -e
for pass in 1 2; do
  for v in "$@"; do
    echo "== $v"
    timeout -k 10 300 python scripts/experiments/texture_ksize_bench.py --lib variants/$v.so ${KS:-7 9 11 13 15}
  done
done
