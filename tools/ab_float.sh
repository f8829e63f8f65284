#!/bin/bash
# A/B of the float fast path (product) vs the uint32-key network for every
# wave (tools/libp2pdl_nofloat.so) on the same box; robust GPU tests first.
set -o pipefail
OUT=${1:-gpurun_out/abfloat}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "robust or dropin" > "$OUT/pytest_robust.log" 2>&1 || { tail -30 "$OUT/pytest_robust.log"; exit 1; }
tail -1 "$OUT/pytest_robust.log"
B="bench.py --no-sub --no-cpu-baseline --steps 10 --warmup 2"
for w in median256 trimmed256 cfg4-median cfg4-trimmed; do
  timeout -k 10 200 python -u $B --workload $w > "$OUT/prod_$w.log" 2>&1 || { tail "$OUT/prod_$w.log"; exit 1; }
  if [ "$w" = median256 ] || [ "$w" = trimmed256 ]; then
    P2P_LIB=tools/libp2pdl_nofloat.so timeout -k 10 200 python -u $B --workload $w > "$OUT/nofloat_$w.log" 2>&1 || { tail "$OUT/nofloat_$w.log"; exit 1; }
  fi
done
grep -h '"kernel_ms"' "$OUT"/*.log | sed 's/.*"workload": "\([^:]*\):.*"frac": \([0-9.]*\).*"kernel_ms": \([0-9.]*\).*/\1 frac=\2 kernel_ms=\3/'
ls "$OUT"
