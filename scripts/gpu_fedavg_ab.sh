#!/bin/bash
# GPU parity tests + FedAvg tile-size A/B (P2P_FEDAVG_NV) on cfg2 and cfg3.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-fedavg_ab}
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -gt 1 ] && exit $rc
for nv in 1 2 4; do
  P2P_FEDAVG_NV=$nv timeout -k 10 120 python bench.py --workload cfg2 --steps 50 --warmup 5 --no-cpu-baseline --no-check > "$OUT/cfg2_nv$nv.log" 2>&1 || exit $?
  tail -1 "$OUT/cfg2_nv$nv.log" | python3 -c "import sys,json; j=json.loads(sys.stdin.read()); print('cfg2 nv=$nv', j['roofline']['kernel_ms'], j['roofline']['frac'])"
done
for nv in 1 4; do
  P2P_FEDAVG_NV=$nv timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check > "$OUT/cfg3_nv$nv.log" 2>&1 || exit $?
  tail -1 "$OUT/cfg3_nv$nv.log" | python3 -c "import sys,json; j=json.loads(sys.stdin.read()); print('cfg3 nv=$nv', j['roofline']['kernel_ms'], j['roofline']['frac'])"
done
