#!/bin/bash
# A/B of library builds with one experiment script, interleaved twice:
#   gpurun -- 'bash scripts/experiments/run_lib_ab.sh <script.py> <lib.so> <lib.so> ... > gpurun_out/x.txt'
# (KS: the ksize list passed to the script)
set -e
script=$1; shift
for pass in 1 2; do
  for v in "$@"; do
    echo "== $v"
    timeout -k 10 300 python $script --lib $v ${KS:-}
  done
done
