#!/bin/bash
# Frames in flight on the SatLut build: C4 and C3 with 2 / 3 streams (no CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c4 c3; do for s in 2 3 2 3; do
  timeout -k 10 200 python bench.py --config $c --streams $s --no-cpu-baseline > gpurun_out/st.json 2>/dev/null || { echo "$c s=$s FAILED"; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/st.json') if l.startswith('{')][-1]); print('$c streams=$s', d['value'], d['ms_per_step'])"
done; done
