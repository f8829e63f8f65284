# Round 6 h: the K = 256 queue question on a second box -- same-process A/B of
# the product (no queue above K = 128) against the queue at K = 256 (q256) and
# no queue at all, plus the standalone lab (P vs Q) on the cfg3 plane shape.
set -o pipefail
O=gpurun_out/r06h; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/lib_pair_ab.py 24 prod q256 noqueue -- 256:16777216 256:7559488 128:16777216 64:100007936 \
  > $O/pair_ab.log 2>&1 || { tail -30 $O/pair_ab.log; exit 1; }
cat $O/pair_ab.log
timeout -k 10 120 tools/split_fixed_lab 256 16777216 15 > $O/lab_k256.log 2>&1 || { tail $O/lab_k256.log; exit 1; }
grep -v bit-exact $O/lab_k256.log
echo done
