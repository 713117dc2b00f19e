set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "fused or texture_end_to_end" --timeout 120 --timeout-method thread > gpurun_out/fused_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -6 gpurun_out/fused_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -k "c4" --timeout 200 --timeout-method thread > gpurun_out/fused_full.log 2>&1
rc=$?; echo "fullsize rc=$rc"; tail -4 gpurun_out/fused_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/variant_bench.py various_image_processings_amd/libvip_hip.so > gpurun_out/fused_timing.log 2>&1
rc=$?; echo "timing rc=$rc"; cat gpurun_out/fused_timing.log; exit $rc
