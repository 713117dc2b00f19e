#!/bin/bash
# GPU parity tests on the current build (optional), then parity + timing of variant
# libraries (variants/*.so), each check under its own time limit.
# usage: gpu_variants.sh [notests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${1:-}" != notests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for so in variants/*.so; do
  timeout -k 10 300 python scripts/variant_parity.py $so >> gpurun_out/variants.log 2>&1
  rc=$?; echo "parity $so rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
timeout -k 10 600 python scripts/variant_bench.py variants/*.so >> gpurun_out/variants.log 2>&1
rc=$?; echo "variants rc=$rc"; cat gpurun_out/variants.log; exit $rc
