#!/bin/bash
# Round 3: bench line + rocprofv3 stats + PMC for the runtime-radius kernel (k65 config),
# and a PMC pass for C1 (its kernel changed to the wide tiles this round).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
# the N > 1 native bench path in one process (one-rank RCCL communicator)
timeout -k 10 200 python bench.py --config c2 --rehearse-native --steps 200 --no-cpu-baseline > gpurun_out/r03_native_rehearsal.json 2> gpurun_out/b_nat.err
rc=$?; echo "native rehearsal rc=$rc"; cat gpurun_out/r03_native_rehearsal.json | grep -v Gloo; [ $rc -eq 0 ] || { tail -20 gpurun_out/b_nat.err; exit $rc; }
timeout -k 10 300 python bench.py --config k65 > gpurun_out/r03_k65_bench.json 2> gpurun_out/b_k65.err
rc=$?; echo "bench k65 rc=$rc"; cut -c1-400 gpurun_out/r03_k65_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/b_k65.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k65 -o run --output-format csv -- python bench.py --config k65 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_k65.log 2>&1
rc=$?; echo "rocprof k65 rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/prof_k65/run_kernel_stats.csv gpurun_out/r03_k65_kernel_stats.csv
for c in k65 c1; do
  bash scripts/gpu_pmc.sh $c || exit $?
  python scripts/pmc_summary.py gpurun_out/pmc_$c gpurun_out/r03_${c}_pmc.json > /dev/null || exit $?
done
timeout -k 10 300 python bench.py --config k65 --no-cpu-baseline > gpurun_out/r03_k65_bench2.json 2> gpurun_out/b_k65.err
rc=$?; echo "bench k65 (with PMC summary) rc=$rc"; cut -c1-300 gpurun_out/r03_k65_bench2.json; exit $rc
