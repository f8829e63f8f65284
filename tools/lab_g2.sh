#!/bin/bash
# Lab A/B: product layout (variant 0) vs two sorter groups per block
# (variant 7) at K = 256 (pruned networks) and K = 200 (generic), median and
# trimmed mean, bit-compared on the device.
set -o pipefail
OUT=${1:-gpurun_out/labg2}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in median trimmed; do
  for k in 256 200; do
    P2P_LIB=tools/libp2pdl_lab.so timeout -k 10 300 python -u tools/lab_robust.py --rule $r --peers $k --variants 0,7 --coords 50000000 > $OUT/lab_${r}_$k.log 2>&1 || { tail -20 $OUT/lab_${r}_$k.log; exit 1; }
    grep -h '^{' $OUT/lab_${r}_$k.log | cut -c1-240
  done
done
