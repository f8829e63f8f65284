#!/bin/bash
# Robust-rule parity + A/B of the K in 65..256 kernel layouts (P2P_ROBUST_IMPL).
set -u
TAG=${1:-robust_ab}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
run() { local name=$1 t=$2; shift 2; local s=$SECONDS
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc $((SECONDS-s))s"; tail -1 "$OUT/$name.log" | python3 -c "import sys,json
l=sys.stdin.read().strip()
try:
  j=json.loads(l); print('   ', j['config']['workload'], 'value', j['value'], 'kernel_ms', j['roofline']['kernel_ms'], 'frac', j['roofline']['frac'])
except Exception: print(l[-600:])"; return $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread || exit $?
fi
for impl in ${IMPLS:-auto lds lds2 lds1 group}; do
  for wl in ${WLS:-median256 trimmed256 cfg4-median cfg4-trimmed}; do
    run "${wl}_$impl" 300 env P2P_ROBUST_IMPL=$impl python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline || exit $?
  done
done
