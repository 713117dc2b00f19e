#!/bin/bash
# rocprofv3 kernel-trace stats for one bench config -> gpurun_out/prof_<cfg>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-c2}
ARGS="--config $CFG"
[ "$CFG" = c4fused ] && ARGS="--config c4 --texture-mode fused"  # C4, guide + JBF in one launch
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$CFG -o run --output-format csv -- python bench.py $ARGS --steps 10 --no-cpu-baseline > gpurun_out/prof_$CFG.log 2>&1
rc=$?; echo "rocprof $CFG rc=$rc"; [ $rc -eq 0 ] || exit $rc
python - "$CFG" <<'PY'
import csv, sys
cfg = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/prof_{cfg}/run_kernel_stats.csv")))
for r in rows[:12]:
    print(f"{float(r['AverageNs'])/1e3:10.1f} us avg  x{r['Calls']:>4}  {r['Percentage']:>6}%  {r['Name'][:90]}")
PY
