# Round 6 b: parity of the restructured split kernel (product and tile-queue
# builds), the queue A/B on bench shapes, and SQ counters of the fixed-cost lab.
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
export PYTHONUNBUFFERED=1
T="python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu"
K="split or chunk or slab_rows or dropin_cfg2 or plain_dicts or devk or abi or zero_size"
timeout -k 10 400 $T -k "$K" > $O/tests_prod.log 2>&1 || { tail -30 $O/tests_prod.log; exit 1; }
tail -2 $O/tests_prod.log
P2P_LIB=tools/libp2pdl_queue.so timeout -k 10 400 $T -k "$K" > $O/tests_queue.log 2>&1 || { tail -30 $O/tests_queue.log; exit 1; }
tail -2 $O/tests_queue.log
timeout -k 10 900 tools/queue_ab.sh $O/ab 2 "cfg3|--workload cfg3" "cfg2|--workload cfg2-dropin" \
  "k64n100m|--workload cfg3 --peers 64 --coords 100007936" "k16n100m|--workload cfg3 --peers 16 --coords 100007936" \
  > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_k64 -o run -- tools/split_fixed_lab 64 100007936 3 > $O/pmc_k64.log 2>&1 || { tail $O/pmc_k64.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_k16 -o run -- tools/split_fixed_lab 16 100007936 3 > $O/pmc_k16.log 2>&1 || { tail $O/pmc_k16.log; exit 1; }

timeout -k 10 300 python -u tools/chunks_ab.py 15 64:1 16:1 64:4 > $O/chunks_ab.log 2>&1 || { tail -30 $O/chunks_ab.log; exit 1; }
cat $O/chunks_ab.log
echo done
