#!/bin/bash
# C5 apron question: does reading the 30-row apron cost time? The
# r=15 slab with and without any HBM tile reads (VIP_ABL_NOLOAD, timing only), then the
# C5 PMC summary of the current build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python scripts/variant_bench.py variants/c5base.so variants/c5noload.so variants/c5base.so variants/c5noload.so --r15 --only=bilateral > gpurun_out/c5_noload.txt 2>&1
rc=$?; echo "variant_bench rc=$rc"; cat gpurun_out/c5_noload.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh c5 || exit $?
python scripts/pmc_summary.py gpurun_out/pmc_c5 gpurun_out/r03_c5_pmc.json > /dev/null || exit $?
echo "pmc done"
