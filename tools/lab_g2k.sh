#!/bin/bash
# Lab: variant 0 vs 7 (two sorter groups) across generic K (MODE 0 paths).
set -o pipefail
OUT=${1:-gpurun_out/labg2k}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in median trimmed; do
  for k in 129 160 224 255; do
    P2P_LIB=tools/libp2pdl_lab.so timeout -k 10 300 python -u tools/lab_robust.py --rule $r --peers $k --variants 0,7 --coords 30000000 --steps 6 > $OUT/lab_${r}_$k.log 2>&1 || { tail -20 $OUT/lab_${r}_$k.log; exit 1; }
    grep -h '^{' $OUT/lab_${r}_$k.log | python3 -c "import sys,json; [print(d['rule'], d['peers'], 'v', d['variant'], d['ms_median'], d['frac_hbm'], d['bit_equal_to_variant0']) for d in map(json.loads, sys.stdin)]"
  done
done
