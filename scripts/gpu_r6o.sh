# Round 6 o: the late-claim queue schedule (qlate, queue up to K = 256) --
# parity on the split / chunk / rows tests, then same-process A/B against the
# product (early claims, K <= 128), the early schedule at K = 256 and no queue.
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
export PYTHONUNBUFFERED=1
P2P_LIB=tools/libp2pdl_qlate.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "(split or chunk or slab_rows or dropin_cfg2 or graph) and not split_plan_takes" > $O/tests_qlate.log 2>&1 || { tail -30 $O/tests_qlate.log; exit 1; }
tail -1 $O/tests_qlate.log
timeout -k 10 700 python -u tools/lib_pair_ab.py 24 prod qlate q256 noqueue -- 256:16777216 256:7559488 64:100007936 16:100007936 rows:64:1 sd:64:1 \
  > $O/pair_ab.log 2>&1 || { tail -30 $O/pair_ab.log; exit 1; }
cat $O/pair_ab.log
echo done
