#!/bin/bash
# Round evidence on one GPU box: the -m gpu suite, smoke, one default bench line per config
# (2 frames in flight, CPU baseline), then rocprofv3 kernel stats + isolated-launch
# durations of the default command per config. Each GPU step has its own limit; a crash,
# fault or timeout ends the script (pytest rc 1 = test failures: reported, not a fault).
# usage: gpu_final.sh [tests|bench|prof|all]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
what=${1:-all}
if [ "$what" = tests ] || [ "$what" = all ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --durations=10 --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
  { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  for c in c2 c3 c4 c5 c1; do
    timeout -k 10 400 python bench.py --config $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
    rc=$?; echo "bench $c rc=$rc"; cut -c1-200 gpurun_out/bench_$c.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$c.err; exit $rc; }
  done
fi
if [ "$what" = prof ] || [ "$what" = all ]; then
  for c in c2 c3 c4 c5 c1; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- \
      python bench.py --config $c --no-cpu-baseline > gpurun_out/prof_$c.json 2> gpurun_out/prof_$c.err
    rc=$?; echo "rocprof $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_$c.err; exit $rc; }
    python scripts/kernel_busy.py gpurun_out/prof_$c/run_kernel_trace.csv gpurun_out/prof_${c}_busy.json > /dev/null
    rm -f gpurun_out/prof_$c/run_kernel_trace.csv
  done
fi
