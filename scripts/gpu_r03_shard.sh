#!/bin/bash
# Round 3: native shard tests, N=1 bench sanity, N=2 one-GPU rehearsals of the new bench
# structure (strong scaling + weak extra; torch P2P over gloo; native -> fallback).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard_native.py -x -v -rf --timeout 200 --timeout-method thread > gpurun_out/shard_native.log 2>&1
rc=$?; echo "shard tests rc=$rc"; tail -25 gpurun_out/shard_native.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --config c2 --steps 200 --no-cpu-baseline > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err
rc=$?; echo "bench c2 rc=$rc"; cut -c1-600 gpurun_out/b_c2.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/b_c2.err; exit $rc; }
port=29611
for cfg in c2 c5; do
  port=$((port+1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --backend gloo --same-device --config $cfg --steps 8 --warmup 1 \
    > gpurun_out/rehearsal_$cfg.json 2> gpurun_out/rehearsal_$cfg.err
  rc=$?; echo "rehearsal $cfg rc=$rc"; cat gpurun_out/rehearsal_$cfg.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/rehearsal_$cfg.err; exit $rc; }
done
# native exchange with two ranks on one GPU: RCCL rejects the duplicate device, every
# rank sees the failure and the run falls back to torch P2P (gloo here), recorded in the line
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port $((port+1)) bench.py --gpus 2 --backend gloo --same-device --exchange native --config c2 --steps 8 \
  --warmup 1 --no-weak > gpurun_out/rehearsal_native_fallback.json 2> gpurun_out/rehearsal_native_fallback.err
rc=$?; echo "native fallback rc=$rc"; cat gpurun_out/rehearsal_native_fallback.json; grep -m5 "bench.py\|rror" gpurun_out/rehearsal_native_fallback.err | cut -c1-300
exit $rc
