#!/bin/bash
# GPU parity tests on the current build, then time variant libraries (variants/*.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python scripts/variant_bench.py variants/*.so > gpurun_out/variants.log 2>&1
rc=$?; echo "variants rc=$rc"; cat gpurun_out/variants.log; exit $rc
