#!/bin/bash
# A/B of the product library against an alternative build on the same box
# (robust + drop-in GPU tests of the product first), interleaved per workload.
#   usage: tools/ab_lib.sh <out-dir under gpurun_out/> <alt .so> [workloads...]
set -o pipefail
OUT=${1:-gpurun_out/ab}; ALT=$2; shift 2
WL=${*:-median256 trimmed256 cfg4-median cfg4-trimmed}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "robust or dropin" > "$OUT/pytest_robust.log" 2>&1 || { tail -30 "$OUT/pytest_robust.log"; exit 1; }
tail -1 "$OUT/pytest_robust.log"
B="bench.py --no-sub --no-cpu-baseline --steps 10 --warmup 2"
for w in $WL; do
  for rep in 1 2; do
    timeout -k 10 200 python -u $B --workload $w > "$OUT/prod${rep}_$w.log" 2>&1 || { tail "$OUT/prod${rep}_$w.log"; exit 1; }
    P2P_LIB=$ALT timeout -k 10 200 python -u $B --workload $w > "$OUT/alt${rep}_$w.log" 2>&1 || { tail "$OUT/alt${rep}_$w.log"; exit 1; }
  done
done
for f in "$OUT"/prod*.log "$OUT"/alt*.log; do
  echo "$(basename $f .log) $(grep -h '"kernel_ms"' $f | sed 's/.*"frac": \([0-9.]*\).*"kernel_ms": \([0-9.]*\).*/frac=\1 kernel_ms=\2/')"
done
