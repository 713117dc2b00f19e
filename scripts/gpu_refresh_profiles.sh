#!/bin/bash
# Round-end evidence on one GPU: bench line per config, rocprofv3 kernel stats per
# config, PMC passes for the configs given in $PMC_CFGS. Each GPU step has its own
# limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c2 c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; cut -c1-300 gpurun_out/bench_$c.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$c.err; exit $rc; }
done
for c in c2 c3 c4 c5; do
  steps=20; [ $c = c5 ] && steps=5
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python bench.py --config $c --steps $steps --warmup 3 --no-cpu-baseline > gpurun_out/prof_$c.log 2>&1
  rc=$?; echo "rocprof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for c in ${PMC_CFGS:-}; do
  bash scripts/gpu_pmc.sh $c || exit $?
  python scripts/pmc_summary.py gpurun_out/pmc_$c gpurun_out/r01_${c}_pmc.json || exit $?
done
