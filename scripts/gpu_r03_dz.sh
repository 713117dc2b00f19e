#!/bin/bash
# Folded JBF SatLut: DZ = 31 (round-3 first build) vs the largest DZ the 16-bit range allows
# (fewer saturated lanes, fewer 2-way conflicts on copy 31's bank); parity first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_ksize.py tests/test_gpu_dropin.py -m gpu -q -x \
  -k "joint or texture or jbf or dropin or vip_filter" --timeout 300 --timeout-method thread > gpurun_out/pytest_dz.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_dz.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/variant_bench.py variants/dz31.so variants/dz63.so variants/dz31.so variants/dz63.so --only=joint_r4_texture --only=texture_k5_nitr5 > gpurun_out/dz_bench.txt 2>&1
rc=$?; echo "variant_bench rc=$rc"; cat gpurun_out/dz_bench.txt
