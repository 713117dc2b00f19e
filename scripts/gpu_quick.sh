#!/bin/bash
# Quick GPU check of the current build: full GPU parity suite, then per-filter 4K timings
# (scripts/variant_bench.py on the in-tree library and on any variants/*.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/variant_bench.py various_image_processings_amd/libvip_hip.so $(ls variants/*.so 2>/dev/null) > gpurun_out/variants.log 2>&1
rc=$?; echo "variants rc=$rc"; cat gpurun_out/variants.log; exit $rc
