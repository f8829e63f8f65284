# Round 6 c: the slot-ring tile queue -- parity (product and queue builds,
# graph replay), a 3-round A/B on bench shapes incl. cfg3_full and the drop-in
# general path, and the chunk-route A/B under the queue build.
set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
export PYTHONUNBUFFERED=1
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu"
K="split or chunk or slab_rows or dropin_cfg2 or plain_dicts or devk or abi or zero_size or graph"
timeout -k 10 400 $T -k "$K" > $O/tests_prod.log 2>&1 || { tail -30 $O/tests_prod.log; exit 1; }
tail -1 $O/tests_prod.log
P2P_LIB=tools/libp2pdl_queue.so timeout -k 10 400 $T -k "$K" > $O/tests_queue.log 2>&1 || { tail -30 $O/tests_queue.log; exit 1; }
tail -1 $O/tests_queue.log
timeout -k 10 780 tools/queue_ab.sh $O/ab 3 "cfg3|--workload cfg3" "full|--job cfg3-full --steps 1" "cfg2|--workload cfg2-dropin" \
  "k16n100m|--workload cfg3 --peers 16 --coords 100007936" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
P2P_LIB=tools/libp2pdl_queue.so timeout -k 10 300 python -u tools/chunks_ab.py 15 64:1 16:1 > $O/chunks_ab_queue.log 2>&1 || { tail -30 $O/chunks_ab_queue.log; exit 1; }
cat $O/chunks_ab_queue.log
echo done
