#!/bin/bash
# Parity tests + smoke + one bench workload + its rocprofv3 kernel stats and
# the two PMC HBM-traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs).
# usage: gpu_profile.sh TAG WORKLOAD KERNEL_SUBSTR COORDS PEERS [extra bench args]
set -u
TAG=${1:-prof}; WL=${2:-cfg3}; KN=${3:-fedavg_flat_kernel}; COORDS=${4:-125000000}; PEERS=${5:-256}
shift 5 || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
run() { local name=$1 t=$2; shift 2; local s=$SECONDS
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc $((SECONDS-s))s"; tail -2 "$OUT/$name.log" | cut -c1-1500; return $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread || exit $?
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
run bench 600 python bench.py --workload "$WL" --steps 10 --warmup 2 "$@" || exit $?
cd /tmp
run stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o bench -- python3 "$ROOT/bench.py" --workload "$WL" --steps 5 --warmup 1 --no-cpu-baseline "$@" || exit $?
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o bench -- python3 "$ROOT/bench.py" --workload "$WL" --steps 2 --warmup 1 --no-cpu-baseline --no-check "$@" || exit $?
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o bench -- python3 "$ROOT/bench.py" --workload "$WL" --steps 2 --warmup 1 --no-cpu-baseline --no-check "$@" || exit $?
python3 "$ROOT/tools/pmc_traffic.py" "$OUT/pmc_fetch" "$OUT/pmc_write" "$KN" "$WL" "$COORDS" "$PEERS" "$OUT/traffic_$WL.json" | tail -8
