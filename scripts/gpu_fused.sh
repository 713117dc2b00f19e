#!/bin/bash
# Fused-texture-mode check: parity (fused cases + texture end-to-end), the C4 4K
# fused == two-launch test, per-filter timings, then bench lines / rocprof / PMC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "texture" --timeout 120 --timeout-method thread > gpurun_out/fused_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/fused_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k "c4" --timeout 200 --timeout-method thread > gpurun_out/fused_full.log 2>&1
rc=$?; echo "fullsize rc=$rc"; tail -3 gpurun_out/fused_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/variant_bench.py various_image_processings_amd/libvip_hip.so > gpurun_out/fused_timing.log 2>&1
rc=$?; echo "timing rc=$rc"; cat gpurun_out/fused_timing.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_fused_evidence.sh
