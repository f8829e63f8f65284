# Round 6 e: flat split launches over every whole tile (alltiles variant)
# against whole CU rounds + the VGPR remainder (product), both with the queue;
# parity of the variant on the split tests first.
set -o pipefail
O=gpurun_out/r06e; mkdir -p $O
export PYTHONUNBUFFERED=1
P2P_LIB=tools/libp2pdl_alltiles.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "(split or devk) and not split_plan_takes" > $O/tests_alltiles.log 2>&1 || { tail -30 $O/tests_alltiles.log; exit 1; }
tail -1 $O/tests_alltiles.log
OTHER=alltiles timeout -k 10 900 tools/queue_ab.sh $O/ab 3 "cfg3|--workload cfg3" "full|--job cfg3-full --steps 1" \
  "k16n100m|--workload cfg3 --peers 16 --coords 100007936" "k64n100m|--workload cfg3 --peers 64 --coords 100007936" \
  > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
echo done
