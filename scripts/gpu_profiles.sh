#!/bin/bash
# Round evidence on one GPU: a bench line per config (with cpu_baseline), rocprofv3
# kernel stats per config, then PMC passes for $PMC_CFGS summarised into
# gpurun_out/<TAG>_<cfg>_pmc.json. Each GPU step has its own limit; the first
# failure ends the script.  usage: TAG=r02 PMC_CFGS="c2 c3 c4 c5" gpu_profiles.sh [configs]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
cfgs=${*:-c1 c2 c3 c4 c5}
for c in $cfgs; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/${TAG}_${c}_bench.json 2> gpurun_out/bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; cut -c1-300 gpurun_out/${TAG}_${c}_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$c.err; exit $rc; }
done
for c in $cfgs; do
  steps=20; [ $c = c5 ] && steps=5
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python bench.py --config $c --steps $steps --warmup 3 --no-cpu-baseline > gpurun_out/prof_$c.log 2>&1
  rc=$?; echo "rocprof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cp gpurun_out/prof_$c/run_kernel_stats.csv gpurun_out/${TAG}_${c}_kernel_stats.csv
done
for c in ${PMC_CFGS:-}; do
  bash scripts/gpu_pmc.sh $c || exit $?
  python scripts/pmc_summary.py gpurun_out/pmc_$c gpurun_out/${TAG}_${c}_pmc.json > /dev/null || exit $?
done
echo "profiles done"
