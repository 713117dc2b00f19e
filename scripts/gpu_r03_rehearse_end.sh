#!/bin/bash
# The N > 1 bench paths on the final round-3 build, on one GPU: 8 gloo ranks sharing cuda:0
# (torch P2P exchange) and the native vip_shard path through a one-rank RCCL communicator.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29655 bench.py --gpus 8 --backend gloo --same-device --config c2 --steps 8 --warmup 1 \
  > gpurun_out/rehearsal8_c2.json 2> gpurun_out/rehearsal8_c2.err
rc=$?; echo "rehearsal n=8 c2 rc=$rc"; cut -c1-600 gpurun_out/rehearsal8_c2.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/rehearsal8_c2.err; exit $rc; }
timeout -k 10 300 python bench.py --rehearse-native --config c2 > gpurun_out/rehearse_native.json 2> gpurun_out/rehearse_native.err
rc=$?; echo "native rehearsal rc=$rc"; cut -c1-600 gpurun_out/rehearse_native.json; [ $rc -eq 0 ] || tail -20 gpurun_out/rehearse_native.err
