#!/bin/bash
# Bench every BASELINE config on one GPU (each under its own time limit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in "$@"; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; cat gpurun_out/bench_$c.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$c.err; exit $rc; }
done
