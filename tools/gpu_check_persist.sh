#!/bin/bash
# Product GPU tests; the persistent-pair lab library through the robust GPU
# tests; then product vs lab on the K = 256 workloads (interleaved, twice).
set -o pipefail
OUT=gpurun_out/chk; mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
P2P_LIB=tools/libp2pdl_persist.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "robust or dropin" > $OUT/pytest_persist.log 2>&1; rc=$?
tail -2 $OUT/pytest_persist.log; [ $rc -eq 0 ] || exit $rc
B="bench.py --no-sub --no-cpu-baseline --steps 10 --warmup 2"
for w in median256 trimmed256; do
  for rep in 1 2; do
    for lib in prod persist; do
      if [ $lib = prod ]; then L=""; else L="P2P_LIB=tools/libp2pdl_$lib.so"; fi
      env $L timeout -k 10 200 python -u $B --workload $w > "$OUT/${lib}${rep}_$w.log" 2>&1 || { tail "$OUT/${lib}${rep}_$w.log"; exit 1; }
      echo "$lib$rep $w $(grep -h '"kernel_ms"' "$OUT/${lib}${rep}_$w.log" | sed 's/.*"frac": \([0-9.]*\).*"kernel_ms": \([0-9.]*\).*/frac=\1 kernel_ms=\2/')"
    done
  done
done
