#!/bin/bash
# Lab: the K = 256 pair kernel with first-round blocks started late (three
# block-selection rules, tools/libp2pdl_st{1,2,3}.so) against the product.
#   usage: tools/lab_stagger.sh <out-dir under gpurun_out/>
set -o pipefail
OUT=${1:-gpurun_out/stagger}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="bench.py --no-sub --no-cpu-baseline --steps 10 --warmup 2"
for w in median256 trimmed256; do
  for lib in prod st1 st2 st3; do
    if [ $lib = prod ]; then L=""; else L="P2P_LIB=tools/libp2pdl_$lib.so"; fi
    env $L timeout -k 10 200 python -u $B --workload $w > "$OUT/${lib}_$w.log" 2>&1 || { tail "$OUT/${lib}_$w.log"; exit 1; }
    echo "$lib $w $(grep -h '"kernel_ms"' "$OUT/${lib}_$w.log" | sed 's/.*"frac": \([0-9.]*\).*"kernel_ms": \([0-9.]*\).*/frac=\1 kernel_ms=\2/')"
  done
done
