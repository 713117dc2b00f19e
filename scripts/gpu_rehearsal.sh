#!/bin/bash
# N>1 rehearsal on a 1-GPU box: 2 ranks, gloo, both on cuda:0 (bench.py --same-device),
# every config; then the host-frame pipeline sample. Each step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
port=29511
for cfg in c2 c3 c4 c5; do
  port=$((port+1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --backend gloo --same-device --config $cfg --steps 8 --warmup 1 \
    > gpurun_out/rehearsal_$cfg.json 2> gpurun_out/rehearsal_$cfg.err
  rc=$?; echo "rehearsal $cfg rc=$rc"; cut -c1-300 gpurun_out/rehearsal_$cfg.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/rehearsal_$cfg.err; exit $rc; }
done
# a failing RCCL rendezvous (two ranks on one GPU: RCCL rejects the duplicate device)
# must end the run with a message and a non-zero status, not hang
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port $((port+1)) bench.py --gpus 2 --backend nccl --same-device --config c2 --steps 4 --warmup 1 \
  > gpurun_out/rehearsal_nccl_fail.json 2> gpurun_out/rehearsal_nccl_fail.err
rc=$?; echo "nccl-on-one-gpu rc=$rc (expected non-zero, not 124/137)"; grep -m3 "process group\|Error\|error" gpurun_out/rehearsal_nccl_fail.err | cut -c1-300
{ [ $rc -eq 124 ] || [ $rc -eq 137 ]; } && exit $rc
timeout -k 10 300 ./samples/vip_host_pipeline 3840 2160 60 15 3 > gpurun_out/host_pipeline.log 2>&1
rc=$?; echo "host pipeline rc=$rc"; cat gpurun_out/host_pipeline.log; exit $rc
