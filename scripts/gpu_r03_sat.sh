#!/bin/bash
# Saturating-address folded JBF LUT (SatLut): the instruction's semantics on gfx950 first
# (microbench/sat_addr), then the joint/texture parity tests, then timing against the
# library built without it (variants/nosat.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 ./microbench/sat_addr > gpurun_out/sat_addr.txt 2>&1
rc=$?; echo "sat_addr rc=$rc"; cat gpurun_out/sat_addr.txt; [ $rc -eq 0 ] || exit $rc
grep -q "v_mad_legacy_u16 clamp.*S=1280.*mismatches 0 / 1024; high16 kept 0, zeroed 1024" gpurun_out/sat_addr.txt || { echo "legacy mad semantics differ: stop"; exit 5; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_ksize.py -m gpu -q -x \
  -k "joint or texture or jbf or adaptive" --timeout 300 --timeout-method thread > gpurun_out/pytest_sat.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_sat.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/variant_bench.py variants/nosat.so various_image_processings_amd/libvip_hip.so > gpurun_out/sat_bench.txt 2>&1
rc=$?; echo "variant_bench rc=$rc"; cat gpurun_out/sat_bench.txt
