#!/bin/bash
# Full GPU suite on the round-4 tree + digest boundary + drop-in records.
set -o pipefail
OUT=${1:-gpurun_out/r4b}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/digest_boundary.py "$OUT/digest_boundary.json" > "$OUT/digest_boundary.log" 2>&1 || { tail -20 "$OUT/digest_boundary.log"; exit 1; }
grep -h '^{' "$OUT/digest_boundary.log"
for w in cfg1 cfg2-dropin; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 50 --warmup 3 --cpu-seconds 2 > "$OUT/$w.log" 2>&1 || { tail -20 "$OUT/$w.log"; exit 1; }
  grep -h '^{' "$OUT/$w.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$w', d['ms_per_step'], c.get('us_per_call'), c.get('us_per_call_general_path'), d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
