#!/bin/bash
# bench.py with frames in flight on 2 streams (default) against --streams 1, every config,
# then the N=2 gloo rehearsal (both ranks on cuda:0) of c2 and c4 with 2 streams.
# Each GPU step has its own limit; a crash / fault / timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in ${CFGS:-c2 c4 c3 c5}; do
  for s in 2 1; do
    timeout -k 10 300 python bench.py --config $c --streams $s --no-cpu-baseline > gpurun_out/bench_${c}_s$s.json 2> gpurun_out/bench_${c}_s$s.err
    rc=$?; echo "bench $c streams=$s rc=$rc"; python -c "
import json,sys; d=json.load(open('gpurun_out/bench_${c}_s$s.json'))
print(d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('frame_ms_in_flight'), d['roofline'].get('frac'))" ; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${c}_s$s.err; exit $rc; }
  done
done
port=29611
for c in c2 c4; do
  port=$((port+1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --backend gloo --same-device --config $c --steps 8 --warmup 2 \
    > gpurun_out/rehearsal_$c.json 2> gpurun_out/rehearsal_$c.err
  rc=$?; echo "rehearsal $c rc=$rc"; cut -c1-400 gpurun_out/rehearsal_$c.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/rehearsal_$c.err; exit $rc; }
done
