#!/bin/bash
# Round 3 validation on one GPU: the whole -m gpu suite and smoke(), then the N>1 bench
# rehearsed with 8 gloo ranks on cuda:0 (c2 strong scaling of the 4K frame + weak figure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --durations=12 --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_r03.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -22 gpurun_out/pytest_gpu_r03.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_r03.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29655 bench.py --gpus 8 --backend gloo --same-device --config c2 --steps 8 --warmup 1 \
  > gpurun_out/rehearsal8_c2.json 2> gpurun_out/rehearsal8_c2.err
rc=$?; echo "rehearsal n=8 c2 rc=$rc"; cat gpurun_out/rehearsal8_c2.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/rehearsal8_c2.err; exit $rc; }
