#!/bin/bash
# Parity (vs oracle) of every variants/*.so, then 4K timings of the in-tree build and the variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in variants/*.so; do
  timeout -k 10 200 python scripts/variant_parity.py $v || exit 1
done
timeout -k 10 300 python scripts/variant_bench.py various_image_processings_amd/libvip_hip.so variants/*.so
