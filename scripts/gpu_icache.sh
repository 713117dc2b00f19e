#!/bin/bash
# Instruction-cache counters for the bilateral kernels (C2 r=7: 67 KB of code, C5 r=15:
# 298 KB). One small counter set per rocprofv3 pass, each under a hard time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in c2 c5; do
  steps=5; [ $cfg = c5 ] && steps=2
  i=0
  for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_INSTS_VALU"; do
    i=$((i+1))
    OUT=gpurun_out/icache_$cfg/p$i
    mkdir -p $OUT
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $OUT -o run --output-format csv -- python bench.py --config $cfg --steps $steps --warmup 1 --settle-s 0 --no-cpu-baseline > $OUT.log 2>&1
    rc=$?; echo "$cfg pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT.log; exit $rc; }
  done
done
python - <<'PY'
import csv, glob, collections
for cfg in ("c2", "c5"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/icache_{cfg}/p*/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("void vip::bilateral_kernel"):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(cfg, {k: round(sum(v) / len(v)) for k, v in sorted(agg.items())})
PY
