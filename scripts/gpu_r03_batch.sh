#!/bin/bash
# vip_shard_run_batch (several frames' halos in one RCCL group): the native shard tests,
# then the N > 1 native bench path through a one-rank communicator (its split x batch trial).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard_native.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_batch.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_batch.log; [ $rc -eq 0 ] || exit $rc
for c in c2 c3; do
  timeout -k 10 300 python bench.py --rehearse-native --config $c --no-cpu-baseline > gpurun_out/rehearse_native_$c.json 2> gpurun_out/rehearse_native_$c.err
  rc=$?; echo "native rehearsal $c rc=$rc"; grep '^{' gpurun_out/rehearse_native_$c.json | cut -c1-200; [ $rc -eq 0 ] || { tail -20 gpurun_out/rehearse_native_$c.err; exit $rc; }
done
