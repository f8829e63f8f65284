# Round 6 x: the whole GPU suite and smoke on the current tree (layout cache, direct exchange)
set -o pipefail
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
# the N = 2 gloo rehearsal: stdout must be exactly the one JSON line
P2P_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --coords 20000000 --steps 5 --warmup 1 --no-cpu-baseline > $O/dist2.json 2> $O/dist2.log || { tail -30 $O/dist2.log; exit 1; }
python -c "
import json; lines=open('$O/dist2.json').read().splitlines(); assert len(lines) == 1, lines[:3]
d=json.loads(lines[0]); print('stdout: one JSON line', d['n_gpus'], d['value'], sorted(d['config']['gather_legs']))"
