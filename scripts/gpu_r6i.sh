# Round 6 i: the rows kernel with the tile queue (qrows) against the product
# (one block per tile for rows), same process; and the chunk list again.
set -o pipefail
O=gpurun_out/r06i; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/lib_pair_ab.py 24 prod qrows noqueue -- rows:64:1 rows:16:1 rows:64:4 sd:64:1 \
  > $O/pair_ab.log 2>&1 || { tail -30 $O/pair_ab.log; exit 1; }
cat $O/pair_ab.log
echo done
