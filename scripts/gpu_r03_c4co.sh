#!/bin/bash
# Round 3: C4 co-scheduling experiment -- JBF variants small enough to share a CU with
# the guide stage of the frame in flight on the other stream; parity first, then the
# per-frame time with 1/2/3 frames in flight.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/c4co.log
for so in variants/*.so; do
  timeout -k 10 300 python scripts/variant_parity.py $so >> gpurun_out/c4co.log 2>&1
  rc=$?; echo "parity $so rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
timeout -k 10 600 python scripts/c4_inflight_bench.py variants/base.so variants/js8.so variants/js16.so variants/j8.so variants/base.so >> gpurun_out/c4co.log 2>&1
rc=$?; echo "inflight rc=$rc"; cat gpurun_out/c4co.log; exit $rc
