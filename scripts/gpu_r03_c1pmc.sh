#!/bin/bash
# C1's PMC summary for the throughput tiling its bench line uses (16-wave 256-px tiles), then the line again.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_pmc.sh c1 || exit $?
python scripts/pmc_summary.py gpurun_out/pmc_c1 gpurun_out/r03_c1_pmc.json > /dev/null || exit $?
cp gpurun_out/r03_c1_pmc.json profiles/r03_c1_pmc.json
timeout -k 10 300 python bench.py --config c1 > gpurun_out/r03_c1_bench.json 2> gpurun_out/bench_c1.err
rc=$?; echo "bench c1 rc=$rc"; cut -c1-300 gpurun_out/r03_c1_bench.json
