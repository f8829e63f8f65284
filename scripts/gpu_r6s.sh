# Round 6 s: the segment-table layout cache -- the whole GPU suite (every
# state_dict path rebuilds or reuses layouts), smoke, and the general path's
# host time with a new table every call (cfg1, cfg2) and the drop-in lines.
set -o pipefail
O=gpurun_out/r06s; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u tools/prof_general.py 100 mlp > $O/prof_mlp.log 2>&1 || { tail $O/prof_mlp.log; exit 1; }
head -3 $O/prof_mlp.log | tail -1
timeout -k 10 300 python -u tools/prof_general.py 30 > $O/prof_r18.log 2>&1 || { tail $O/prof_r18.log; exit 1; }
head -3 $O/prof_r18.log | tail -1
for w in cfg1 cfg2-dropin; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-reference-gpu > $O/$w.json 2> $O/$w.err || { tail $O/$w.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$w.json').readline()); print('$w', d['ms_per_step'], d.get('general_path'))"
done
echo done
