#!/bin/bash
# Round 3 re-entry: the whole -m gpu suite, smoke() and the default bench line on the rebuilt tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 60 ./microbench/sat_addr > gpurun_out/sat_addr.txt 2>&1; echo "sat_addr rc=$?"; cat gpurun_out/sat_addr.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --durations=12 --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r03b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -22 gpurun_out/pytest_gpu_r03b.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03b.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_r03b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_default.json; [ $rc -eq 0 ] || tail -20 gpurun_out/bench_default.err
