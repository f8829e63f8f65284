# Round 6 d: the whole GPU suite on the queue default, smoke, the gloo N=2
# rehearsal (per-rank pipeline fields, both all-gather legs) and the default
# bench line (cfg5 / cfg5-arrival bounds, the drop-in's general path).
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
P2P_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --coords 20000000 \
  --no-cpu-baseline > $O/dist2.log 2>&1 || { tail -30 $O/dist2.log; exit 1; }
grep -h '^{' $O/dist2.log > $O/dist2.json
cut -c1-1500 $O/dist2.json
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-3000 $O/bench.json
echo done
