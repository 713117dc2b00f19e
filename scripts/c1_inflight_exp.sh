#!/bin/bash
# C1 (lenna 512^2, 10.7 us per launch): frames in flight vs tile shape and stream count
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # label env... -- bench args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 120 python bench.py --config c1 --no-cpu-baseline "$@" > gpurun_out/c1x.json 2>/dev/null || { echo "$label FAILED"; return 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/c1x.json') if l.startswith('{')][-1]); print('$label', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}
run auto_s2 X=1 -- --streams 2
run auto_s4 X=1 -- --streams 4
run w16_s2 VIP_BIL_WAVES=16 VIP_BIL_WIDE=2 -- --streams 2
run w16_s3 VIP_BIL_WAVES=16 VIP_BIL_WIDE=2 -- --streams 3
run w16_s4 VIP_BIL_WAVES=16 VIP_BIL_WIDE=2 -- --streams 4
run w16_s6 VIP_BIL_WAVES=16 VIP_BIL_WIDE=2 -- --streams 6
run n16_s4 VIP_BIL_WAVES=16 VIP_BIL_WIDE=1 -- --streams 4
run n16_s6 VIP_BIL_WAVES=16 VIP_BIL_WIDE=1 -- --streams 6
run w8_s4 VIP_BIL_WAVES=8 VIP_BIL_WIDE=2 -- --streams 4
run w8_s6 VIP_BIL_WAVES=8 VIP_BIL_WIDE=2 -- --streams 6
run n8_s6 VIP_BIL_WAVES=8 VIP_BIL_WIDE=1 -- --streams 6
