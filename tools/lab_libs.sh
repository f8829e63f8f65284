#!/bin/bash
# Lab: bench workloads on the product library and on lab builds (no parity
# tests; lab builds may compute wrong results on purpose, hence --no-check).
#   usage: tools/lab_libs.sh <out-dir under gpurun_out/> "<lib tags>" "<workloads>"
#   tag "prod" = the product library, tag X = tools/libp2pdl_X.so
set -o pipefail
OUT=${1:-gpurun_out/lab}; LIBS=${2:-prod}; WL=${3:-median256 trimmed256}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="bench.py --no-sub --no-cpu-baseline --no-check --steps 10 --warmup 2"
for w in $WL; do
  for lib in $LIBS; do
    if [ $lib = prod ]; then L=""; else L="P2P_LIB=tools/libp2pdl_$lib.so"; fi
    env $L timeout -k 10 200 python -u $B --workload $w > "$OUT/${lib}_$w.log" 2>&1 || { tail "$OUT/${lib}_$w.log"; exit 1; }
    echo "$lib $w $(grep -h '"kernel_ms"' "$OUT/${lib}_$w.log" | sed 's/.*"frac": \([0-9.]*\).*"kernel_ms": \([0-9.]*\).*/frac=\1 kernel_ms=\2/')"
  done
done
