#!/bin/bash
# Padded robust kernels: the robust GPU tests, then the off-config K benches.
set -o pipefail
OUT=gpurun_out/pad; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "robust or median or trim or pair" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for w in median200 trimmed200 median96 trimmed96 median256 trimmed256 cfg4-median cfg4-trimmed; do
  timeout -k 10 200 python -u bench.py --no-sub --no-cpu-baseline --steps 5 --warmup 1 --workload $w > $OUT/$w.log 2>&1 || { tail -5 $OUT/$w.log; exit 1; }
  grep -h "spot check" $OUT/$w.log
  grep -h kernel_ms $OUT/$w.log | sed "s/.*\"frac\": \([0-9.]*\).*\"kernel_ms\": \([0-9.]*\).*/$w frac=\1 kernel_ms=\2/"
done
