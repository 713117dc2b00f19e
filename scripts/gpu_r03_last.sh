#!/bin/bash
# Final round-3 state: whole -m gpu suite, smoke(), default bench line, N = 8 gloo rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_last.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_last.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_last.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_last.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_last.json 2> gpurun_out/bench_last.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/bench_last.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29655 bench.py --gpus 8 --backend gloo --same-device --config c2 --steps 8 --warmup 1 \
  > gpurun_out/rehearsal8_last.json 2> gpurun_out/rehearsal8_last.err
rc=$?; echo "rehearsal n=8 rc=$rc"; cut -c1-200 gpurun_out/rehearsal8_last.json; [ $rc -eq 0 ] || tail -5 gpurun_out/rehearsal8_last.err
