#!/bin/bash
# Lab: variants 0 / 7 / 8 (two sorter groups, barrier vs LDS-counter sync),
# small size first (a broken sync shows as a slow, wrong small run), then
# K = 256 and K = 200 at 50M coordinates; bit-compared with variant 0.
set -o pipefail
OUT=${1:-gpurun_out/labg2a}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
P2P_LIB=tools/libp2pdl_lab.so timeout -k 10 60 python -u tools/lab_robust.py --rule median --peers 256 --variants 0,8 --coords 1000000 --steps 3 > $OUT/small.log 2>&1 || { tail -20 $OUT/small.log; exit 1; }
grep -h '^{' $OUT/small.log | cut -c1-230
grep -q '"variant": 8.*"bit_equal_to_variant0": true' $OUT/small.log || { echo "variant 8 wrong at small size"; exit 1; }
for r in median trimmed; do
  for k in 256 200; do
    P2P_LIB=tools/libp2pdl_lab.so timeout -k 10 200 python -u tools/lab_robust.py --rule $r --peers $k --variants 0,7,8 --coords 50000000 --steps 6 > $OUT/lab_${r}_$k.log 2>&1 || { tail -20 $OUT/lab_${r}_$k.log; exit 1; }
    grep -h '^{' $OUT/lab_${r}_$k.log | python3 -c "import sys,json; [print(d['rule'], d['peers'], 'v', d['variant'], d['ms_median'], d['frac_hbm'], d['bit_equal_to_variant0']) for d in map(json.loads, sys.stdin)]"
  done
done
