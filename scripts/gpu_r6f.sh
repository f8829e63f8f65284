# Round 6 f: the share hint + every-whole-tile queue default -- parity
# (split / chunk / share / graph / sharded world-2 GPU tests), the default
# line, and the product against the no-queue build on cfg3 and the full job.
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_sharded.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "split or chunk or slab_rows or dropin_cfg2 or plain_dicts or devk or abi or zero_size or graph or world or planes or nccl" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-1200 $O/bench.json
OTHER=noqueue timeout -k 10 600 tools/queue_ab.sh $O/ab 2 "cfg3|--workload cfg3" "full|--job cfg3-full --steps 1" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
echo done
