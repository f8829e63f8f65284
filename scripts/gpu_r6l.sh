# Round 6 l: the flat VGPR rest in quarter tiles below 4 tiles per CU
# (quarters4) against the product -- parity on the split tests, then the
# same-process A/B on the cfg3 short plane and the full plane.
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O
export PYTHONUNBUFFERED=1
P2P_LIB=tools/libp2pdl_quarters4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "split_kernel or fedavg_vs_oracle or unaligned" > $O/tests_q4.log 2>&1 || { tail -30 $O/tests_q4.log; exit 1; }
tail -1 $O/tests_q4.log
timeout -k 10 600 python -u tools/lib_pair_ab.py 30 prod quarters4 -- 256:7559488 256:16777216 256:15625000 \
  > $O/pair_ab.log 2>&1 || { tail -30 $O/pair_ab.log; exit 1; }
cat $O/pair_ab.log
echo done
