#!/bin/bash
# Round 6: the split kernel's per-tile fixed cost (tools/split_fixed_lab.hip).
# usage: tools/gpu_fixed_lab.sh <out> "K n" ...
set -o pipefail
OUT=gpurun_out/${1:-fixed_lab}; shift; mkdir -p $OUT
L=tools/split_fixed_lab
for a in "$@"; do
  set -- $a
  timeout -k 10 120 $L $1 $2 ${3:-15} > $OUT/K$1_n$2.log 2>&1 || { echo "FAIL K=$1 n=$2"; tail $OUT/K$1_n$2.log; exit 1; }
  grep -v bit-exact $OUT/K$1_n$2.log
done
