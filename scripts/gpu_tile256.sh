#!/bin/bash
# K <= 128 kernels on 256-coordinate blocks: robust GPU tests, then an
# interleaved A/B against the 128-coordinate build.
set -o pipefail
OUT=gpurun_out/t256; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "robust or median or trim or pair or sharded or dropin" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="bench.py --no-sub --no-cpu-baseline --steps 10 --warmup 2"
for w in cfg4-median cfg4-trimmed median96 trimmed96 median32; do
  for rep in 1 2; do
    timeout -k 10 200 python -u $B --workload $w > $OUT/t256_${rep}_$w.log 2>&1 || { tail -5 $OUT/t256_${rep}_$w.log; exit 1; }
    P2P_LIB=tools/libp2pdl_tile128.so timeout -k 10 200 python -u $B --workload $w > $OUT/t128_${rep}_$w.log 2>&1 || { tail -5 $OUT/t128_${rep}_$w.log; exit 1; }
  done
done
for f in $OUT/t*.log; do echo "$(basename $f .log) $(grep -h '"kernel_ms"' $f | sed 's/.*"frac": \([0-9.]*\).*"kernel_ms": \([0-9.]*\).*/frac=\1 kernel_ms=\2/')"; done
