#!/bin/bash
# Lab A/B: product layout (variant 0) vs the self-staged layout (variant 6)
# for the K = 256 median and trimmed mean, bit-compared on the device.
set -o pipefail
OUT=${1:-gpurun_out/labself}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in median trimmed; do
  P2P_LIB=tools/libp2pdl_lab.so timeout -k 10 300 python -u tools/lab_robust.py --rule $r --peers 256 --variants 0,6 > $OUT/lab_$r.log 2>&1 || { tail -20 $OUT/lab_$r.log; exit 1; }
  grep -h '^{' $OUT/lab_$r.log
done
