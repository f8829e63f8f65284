#!/bin/bash
# Robust-rule parity + A/B of the K=128 kernel layouts + K=256.
set -u
TAG=${1:-robust}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
run() { local name=$1 t=$2; shift 2; local s=$SECONDS
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc $((SECONDS-s))s"; tail -1 "$OUT/$name.log" | python3 -c "import sys,json
l=sys.stdin.read().strip()
try:
  j=json.loads(l); print(j['config']['workload'], 'value', j['value'], 'kernel_ms', j['roofline']['kernel_ms'], 'frac', j['roofline']['frac'])
except Exception: print(l[-400:])"; return $rc; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -rf; rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
run med128_group 600 python bench.py --workload cfg4-median --steps 5 --warmup 1 --no-cpu-baseline || exit $?
run med128_single 600 env P2P_ROBUST_SINGLE_LANE=1 python bench.py --workload cfg4-median --steps 5 --warmup 1 --no-cpu-baseline || exit $?
run trim128_group 600 python bench.py --workload cfg4-trimmed --steps 5 --warmup 1 --no-cpu-baseline || exit $?
run trim128_single 600 env P2P_ROBUST_SINGLE_LANE=1 python bench.py --workload cfg4-trimmed --steps 5 --warmup 1 --no-cpu-baseline || exit $?
run med256 600 python bench.py --workload median256 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
run trim256 600 python bench.py --workload trimmed256 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
