#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel stats.
# Every GPU step has its own time limit; a crash/fault/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }   # 1 = test failures, not a fault
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --durations=10 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_c2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./samples/vip_benchmark 3840 2160 10 15 5 5 > gpurun_out/sample.log 2>&1
rc=$?; echo "sample rc=$rc"; cat gpurun_out/sample.log | tail -6; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python bench.py --steps 10 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof_c2 -name "*stats*" | head
[ $rc -eq 0 ] || exit $rc
for cfg in c3 c4 c5; do
  timeout -k 10 400 python bench.py --config $cfg --steps 10 --warmup 2 > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err
  rc=$?; echo "bench $cfg rc=$rc"; cut -c1-400 gpurun_out/bench_$cfg.json; [ $rc -eq 0 ] || exit $rc
done
for cfg in c3 c4; do bash scripts/gpu_prof_cfg.sh $cfg || exit $?; done
