#!/bin/bash
# Round-2 GPU session: the full -m gpu suite, smoke, then one bench line per config.
# Every GPU step has its own time limit; a crash / fault / timeout stops the script
# (rc 1 from pytest = test failures, reported, not a fault).
# usage: gpu_r02.sh [tests|bench|all] [bench configs...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
what=${1:-all}; shift || true
cfgs=${*:-c2 c3 c4 c5 c1}
if [ "$what" = tests ] || [ "$what" = all ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --durations=15 --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -15
  { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  for c in $cfgs; do
    timeout -k 10 400 python bench.py --config $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
    rc=$?; echo "bench $c rc=$rc"; cut -c1-600 gpurun_out/bench_$c.json
    [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$c.err; exit $rc; }
  done
fi
