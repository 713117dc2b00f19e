#!/bin/bash
# Round 3, SatLut build: the whole -m gpu suite, smoke(), the default bench line, then the
# C3 / C4 evidence (bench lines, rocprofv3 stats, PMC) for the kernels SatLut changed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --durations=12 --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r03c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -22 gpurun_out/pytest_gpu_r03c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03c.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_r03c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench_default.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_default.err; exit $rc; }
TAG=r03 PMC_CFGS="c3 c4" bash scripts/gpu_profiles.sh c3 c4
