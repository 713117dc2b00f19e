#!/bin/bash
# Round 3 end state: the whole -m gpu suite, smoke(), then a bench line + rocprofv3 stats per
# config (C4's PMC summary from the same kernels is committed: profiles/r03_c4_pmc.json).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --durations=12 --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r03d.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_r03d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03d.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_r03d.log; [ $rc -eq 0 ] || exit $rc
TAG=r03 PMC_CFGS="" bash scripts/gpu_profiles.sh c1 c2 c3 c4 c5
