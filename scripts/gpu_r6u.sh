# Round 6 u: the direct exchange (sharded.exchange_ p2p): the sharded GPU
# tests, then the gloo rehearsal of the N = 2 line (ranks share the one GPU)
# carrying all three exchange legs.
set -o pipefail
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_sharded.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/sharded.log 2>&1 || { tail -30 $O/sharded.log; exit 1; }
tail -3 $O/sharded.log
P2P_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --coords 20000000 --steps 5 --warmup 1 --no-cpu-baseline > $O/dist2.json 2> $O/dist2.log || { tail -30 $O/dist2.log; exit 1; }
python -c "
import json; d=json.loads(open('$O/dist2.json').readline())
print(d['n_gpus'], d['value'], d['ms_per_step'])
for k, v in d['config']['gather_legs'].items(): print(k, json.dumps(v)[:400])
"
echo done
