#!/bin/bash
# The one parametrised GPU runner (round 4 on; it replaces the per-round gpu_r0x_*.sh
# wrappers). Run through gpurun from the repo root:
#
#   TAG=r04 bash scripts/gpu.sh STEP [STEP ...]
#
# Every step runs under its own time limit; the first failing step ends the run, and no
# GPU step follows a fault, abort or timeout. Outputs go to gpurun_out/ (copy what is to
# be judged into profiles/).
#
# STEP
#   tests[=ARGS]        python -m pytest -m gpu ARGS (default: tests, the whole GPU suite; ARGS is
#                       shell-quoted, e.g. tests="tests/test_gpu_parity.py -k 'texture or gradient'")
#   smoke               __graft_entry__.smoke()
#   bench=CFG[,A,..]    bench line              -> ${TAG}_CFG_bench.json (A: extra bench.py args)
#   stats=CFG[,A,..]    rocprofv3 --kernel-trace --stats of a short bench run
#                                               -> ${TAG}_CFG_kernel_stats.csv, ${TAG}_CFG_busy.json
#   iso=CFG[,A,..]      rocprofv3 --kernel-trace of a one-stream, one-frame-per-launch bench run: the last
#                       300 launches of each filter kernel -> ${TAG}_CFG_isolated.csv
#   pmc=CFG[,A,..]      one rocprofv3 --pmc pass per counter set -> ${TAG}_CFG_pmc.json
#   rehearse=CFG,N[,A]  the N > 1 native path on one GPU: bench.py --rehearse-native --loopback N A..
#                                               -> ${TAG}_CFG_loopbackN.json
#   gloo=CFG,N          python bench.py --gpus N --same-device --backend gloo (N ranks on cuda:0)
#                                               -> ${TAG}_CFG_gloo{N}.json
#   py=SCRIPT[,A,..]    python SCRIPT A..       -> ${TAG}_<script name>.txt
#                       (the one-off measurements behind DESIGN.md's tables: scripts/experiments/)
#   variants            variant libraries (variants/*.so from build_variant.sh / build_texture_variant.sh):
#                       parity against the oracle, then timing -> ${TAG}_variants.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${TAG:-r06}
O=gpurun_out

fail() { echo "step '$1' failed rc=$2"; [ -n "${3:-}" ] && tail -25 "$3"; exit "$2"; }

# counter sets, one rocprofv3 pass each (at most 8 SQ_, 4 TCC_ per pass)
PMC_SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
          "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
          "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE"
          "FETCH_SIZE" "WRITE_SIZE")

for step in "$@"; do
  name=${step%%=*}
  arg=""; [ "$step" != "$name" ] && arg=${step#*=}
  IFS=, read -r -a A <<< "$arg"
  echo "== $step"
  case $name in
    tests)
      log=$O/${TAG}_pytest_gpu.log
      eval "timeout -k 10 1100 python -u -m pytest ${arg:-tests} -m gpu -v -x -rf --durations=15 --timeout 300 \
        --timeout-method thread" > $log 2>&1
      rc=$?; tail -8 $log; [ $rc -eq 0 ] || fail "$step" $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1
      rc=$?; tail -2 $O/${TAG}_smoke.log; [ $rc -eq 0 ] || fail "$step" $rc $O/${TAG}_smoke.log ;;
    bench)
      cfg=${A[0]}; out=$O/${TAG}_${cfg}_bench.json
      timeout -k 10 400 python bench.py --config $cfg "${A[@]:1}" > $out 2> $O/${TAG}_${cfg}_bench.err
      rc=$?; cut -c1-600 $out; [ $rc -eq 0 ] || fail "$step" $rc $O/${TAG}_${cfg}_bench.err ;;
    stats)
      cfg=${A[0]}; steps=20; [ $cfg = c5 ] && steps=5; d=$O/prof_${TAG}_$cfg
      # one stream and a 1 s settle: the summary's average is then a launch duration (with two
      # streams the launches overlap and the settle's queued frames dominate the count)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
        python bench.py --config $cfg --steps $steps --warmup 3 --no-cpu-baseline --streams 1 --batch 1 \
        --settle-s 1 "${A[@]:1}" > $d.log 2>&1
      rc=$?; [ $rc -eq 0 ] || fail "$step" $rc $d.log
      cp $d/run_kernel_stats.csv $O/${TAG}_${cfg}_kernel_stats.csv
      python scripts/kernel_busy.py $d/run_kernel_trace.csv $O/${TAG}_${cfg}_busy.json > /dev/null || fail "$step" $?
      rm -rf $d
      head -4 $O/${TAG}_${cfg}_kernel_stats.csv | cut -c1-200 ;;
    iso)
      # step counts are multiples of 12, so a --batch B run (B | 12) has no partial batch whose
      # multi-frame launch would carry fewer frames
      cfg=${A[0]}; steps=1200; [ $cfg = c5 ] && steps=240; [ $cfg = c4 ] && steps=300; [ $cfg = c2 ] && steps=408
      [ $cfg = c3 ] && steps=408; d=$O/iso_${TAG}_$cfg
      timeout -k 10 500 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- \
        python bench.py --config $cfg --streams 1 --batch 1 --steps $steps --warmup 12 --no-cpu-baseline \
        "${A[@]:1}" > $d.log 2>&1
      rc=$?; [ $rc -eq 0 ] || fail "$step" $rc $d.log
      fpl=1; for ((j = 1; j < ${#A[@]}; ++j)); do [ "${A[$j]}" = --batch ] && fpl=${A[$((j + 1))]}; done
      python scripts/isolated_sample.py $d/run_kernel_trace.csv $O/${TAG}_${cfg}_isolated.csv --last 300 \
        --frames-per-launch $fpl || fail "$step" $?
      rm -rf $d ;;  # the raw trace (tens of MB for a small frame) stays on the box
    pmc)
      cfg=${A[0]}; d=$O/pmc_${TAG}_$cfg; mkdir -p $d; i=0
      for set in "${PMC_SETS[@]}"; do
        i=$((i+1))
        timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set -d $d/p$i -o run --output-format csv -- \
          python bench.py --config $cfg --streams 1 --batch 1 --steps 12 --warmup 12 --settle-s 0.3 --no-cpu-baseline \
          "${A[@]:1}" > $d/p$i.log 2>&1
        rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || fail "$step pass $i" $rc $d/p$i.log
      done
      fpl=1; for ((j = 1; j < ${#A[@]}; ++j)); do [ "${A[$j]}" = --batch ] && fpl=${A[$((j + 1))]}; done
      python scripts/pmc_summary.py $d $O/${TAG}_${cfg}_pmc.json --frames-per-launch $fpl | cut -c1-400 || fail "$step" $?
      rm -rf $d/p*/ ;;  # the per-dispatch counter tables stay on the box
    rehearse)
      cfg=${A[0]}; n=${A[1]}; sfx=$(printf '%s' "${A[*]:2}" | tr -c 'a-zA-Z0-9' '_'); out=$O/${TAG}_${cfg}_loopback$n$sfx.json
      timeout -k 10 400 python bench.py --config $cfg --rehearse-native --loopback $n --steps 400 "${A[@]:2}" \
        > $out 2> ${out%.json}.err
      rc=$?; cut -c1-1500 $out; [ $rc -eq 0 ] || fail "$step" $rc ${out%.json}.err ;;
    gloo)
      cfg=${A[0]}; n=${A[1]}; out=$O/${TAG}_${cfg}_gloo$n.json
      timeout -k 10 500 python bench.py --gpus $n --same-device --backend gloo --config $cfg --steps 8 \
        --warmup 1 "${A[@]:2}" > $out 2> $O/${TAG}_${cfg}_gloo$n.err
      rc=$?; cut -c1-800 $out; [ $rc -eq 0 ] || fail "$step" $rc $O/${TAG}_${cfg}_gloo$n.err ;;
    py)
      s=${A[0]}; out=$O/${TAG}_$(basename ${s%.*}).txt
      timeout -k 10 600 python $s "${A[@]:1}" > $out 2>&1
      rc=$?; tail -30 $out; [ $rc -eq 0 ] || fail "$step" $rc ;;
    variants)
      log=$O/${TAG}_variants.log; : > $log
      for so in variants/*.so; do
        timeout -k 10 300 python scripts/variant_parity.py $so >> $log 2>&1
        rc=$?; echo "parity $so rc=$rc"; [ $rc -eq 0 ] || fail "$step parity $so" $rc $log
      done
      timeout -k 10 600 python scripts/variant_bench.py variants/*.so >> $log 2>&1
      rc=$?; tail -30 $log; [ $rc -eq 0 ] || fail "$step" $rc ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu.sh: all steps done"
