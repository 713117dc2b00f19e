#!/bin/bash
# C4 FUSED-mode evidence: bench lines of both modes, rocprofv3 kernel stats and PMC of
# the fused kernel (each GPU step with its own time limit; stop at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mode in two-launch fused; do
  timeout -k 10 300 python bench.py --config c4 --texture-mode $mode --no-cpu-baseline > gpurun_out/bench_c4_$mode.json 2> gpurun_out/bench_c4_$mode.err
  rc=$?; echo "bench c4 $mode rc=$rc"; cut -c1-300 gpurun_out/bench_c4_$mode.json; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_prof_cfg.sh c4fused || exit $?
bash scripts/gpu_pmc.sh c4fused || exit $?
python scripts/pmc_summary.py gpurun_out/pmc_c4fused gpurun_out/r02_c4fused_pmc.json
