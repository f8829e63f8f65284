#!/bin/bash
# Median pair kernel with three wave pairs per block: median GPU tests, then
# an interleaved A/B against the two-pair build.
set -o pipefail
OUT=gpurun_out/np3; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "median or robust" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="bench.py --no-sub --no-cpu-baseline --steps 10 --warmup 2"
for w in median256 median200; do
  for rep in 1 2; do
    timeout -k 10 200 python -u $B --workload $w > $OUT/np3_${rep}_$w.log 2>&1 || { tail -5 $OUT/np3_${rep}_$w.log; exit 1; }
    P2P_LIB=tools/libp2pdl_np2.so timeout -k 10 200 python -u $B --workload $w > $OUT/np2_${rep}_$w.log 2>&1 || { tail -5 $OUT/np2_${rep}_$w.log; exit 1; }
  done
done
for f in $OUT/np*.log; do echo "$(basename $f .log) $(grep -h '"kernel_ms"' $f | sed 's/.*"frac": \([0-9.]*\).*"kernel_ms": \([0-9.]*\).*/frac=\1 kernel_ms=\2/')"; done
