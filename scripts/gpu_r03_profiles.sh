#!/bin/bash
# Round-3 evidence: bench line per config (TAG=r03), rocprofv3 kernel stats per config,
# PMC passes for $PMC_CFGS, and the large-ksize kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r03 PMC_CFGS="${PMC_CFGS:-c2}" bash scripts/gpu_profiles.sh ${*:-c1 c2 c3 c4 c5} || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ksize -o run --output-format csv -- python scripts/ksize_bench.py > gpurun_out/prof_ksize.log 2>&1
rc=$?; echo "rocprof ksize rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/prof_ksize/run_kernel_stats.csv gpurun_out/r03_ksize_kernel_stats.csv
tail -3 gpurun_out/prof_ksize.log
