#!/bin/bash
# rocprofv3 kernel trace + stats of the default bench command per config (2 streams,
# single-stream roofline phase after the timed region), then per-kernel isolated-launch
# durations and device busy time (scripts/kernel_busy.py). usage: gpu_prof_streams.sh [cfgs]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${*:-c2 c4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- \
    python bench.py --config $c > gpurun_out/prof_$c.json 2> gpurun_out/prof_$c.err
  rc=$?; echo "rocprof bench $c rc=$rc"; cut -c1-300 gpurun_out/prof_$c.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_$c.err; exit $rc; }
  python scripts/kernel_busy.py gpurun_out/prof_$c/run_kernel_trace.csv gpurun_out/prof_${c}_busy.json | head -30
done
