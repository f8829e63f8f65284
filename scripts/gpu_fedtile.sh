#!/bin/bash
# FedAvg 2048-float tiles for segment tables and small flat problems: the
# FedAvg / drop-in GPU tests, then an interleaved A/B against 4096-float tiles.
set -o pipefail
OUT=gpurun_out/fedtile; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "fedavg or dropin or segment or golden or fused or inbox" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="bench.py --no-sub --no-cpu-baseline --steps 20 --warmup 3"
for w in cfg2 cfg2-dropin; do
  for rep in 1 2; do
    timeout -k 10 200 python -u $B --workload $w > $OUT/t2048_${rep}_$w.log 2>&1 || { tail -5 $OUT/t2048_${rep}_$w.log; exit 1; }
    P2P_LIB=tools/libp2pdl_fed4.so timeout -k 10 200 python -u $B --workload $w > $OUT/t4096_${rep}_$w.log 2>&1 || { tail -5 $OUT/t4096_${rep}_$w.log; exit 1; }
  done
done
for f in $OUT/t*.log; do echo "$(basename $f .log) $(grep -h '"kernel_ms"' $f | sed 's/.*"frac": \([0-9.]*\).*"kernel_ms": \([0-9.]*\).*/frac=\1 kernel_ms=\2/')"; done
