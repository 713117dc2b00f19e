#!/bin/bash
# PMC counter passes for one bench config (separate passes, kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFG=${1:-c2}
ARGS="--config $CFG"
[ "$CFG" = c4fused ] && ARGS="--config c4 --texture-mode fused"  # C4, guide + JBF in one launch
OUT=gpurun_out/pmc_${CFG}
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- python bench.py $ARGS --streams 1 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
