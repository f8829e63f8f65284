# Round 6 p: the product with late claims (queue to K = 256, every whole
# tile to K = 128) -- parity subset, then same-process A/B against late
# claims to K = 128 (q128), the early schedule (qearly) and no queue.
set -o pipefail
O=gpurun_out/r06p; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_sharded.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "split or chunk or slab_rows or dropin_cfg2 or plain_dicts or devk or graph or world or planes or share" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 800 python -u tools/lib_pair_ab.py 24 prod q128 qearly noqueue -- 256:16777216 256:7559488 256:15625000 64:100007936 16:11689984 rows:64:1 sd:64:1 \
  > $O/pair_ab.log 2>&1 || { tail -30 $O/pair_ab.log; exit 1; }
cat $O/pair_ab.log
echo done
