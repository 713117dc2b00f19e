#!/bin/bash
# After a guide-stage change: the texture GPU tests, the C4 bench line, rocprofv3 stats of the
# default C4 command and the C4 PMC passes. Each GPU step has its own limit; the first
# failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -k "texture or guide or smoke or stream" --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_gpu_tex.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_tex.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config c4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
rc=$?; echo "bench c4 rc=$rc"; cut -c1-200 gpurun_out/bench_c4.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python bench.py --config c4 --no-cpu-baseline > gpurun_out/prof_c4.json 2> gpurun_out/prof_c4.err
rc=$?; echo "rocprof c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/kernel_busy.py gpurun_out/prof_c4/run_kernel_trace.csv gpurun_out/prof_c4_busy.json > /dev/null
rm -f gpurun_out/prof_c4/run_kernel_trace.csv
bash scripts/gpu_pmc.sh c4 || exit $?
python scripts/pmc_summary.py gpurun_out/pmc_c4 gpurun_out/r02_c4_pmc.json
