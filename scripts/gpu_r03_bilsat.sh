#!/bin/bash
# Plain bilateral on the 512 x 32 saturating-address LUT (VIP_BIL_SAT): parity of the
# plain-filter tests, then timing against variants/bilsat0.so (same build, VIP_BIL_SAT=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_ksize.py tests/test_gpu_sharded.py -m gpu -q -x \
  -k "bilateral or c2 or c5 or plain" --timeout 300 --timeout-method thread > gpurun_out/pytest_bilsat.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_bilsat.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/variant_bench.py variants/bilsat0.so variants/bilsat1.so variants/bilsat0.so variants/bilsat1.so --r15 --only=bilateral > gpurun_out/bilsat_bench.txt 2>&1
rc=$?; echo "variant_bench rc=$rc"; cat gpurun_out/bilsat_bench.txt
