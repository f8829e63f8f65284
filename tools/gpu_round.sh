#!/bin/bash
# One gpurun call: GPU parity tests, smoke, the default bench line and a
# rocprofv3 kernel-stats pass over it.  Every GPU step has its own time limit
# and the chain stops at the first failure (no retries).
#   usage: tools/gpu_round.sh <out-dir under gpurun_out/> [pytest -k expr]
set -o pipefail
OUT=${1:-gpurun_out/round}
KEXPR=${2:-}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1

run() {  # run <seconds> <log> <cmd...>
  local secs=$1 logf=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$logf" 2>&1
  local rc=$?
  echo "== rc=$rc" | tee -a "$OUT/steps.log"
  [ $rc -eq 0 ] || { tail -40 "$logf"; exit $rc; }
}

if [ -n "$KEXPR" ]; then
  run 1100 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$KEXPR"
else
  run 1100 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
fi
tail -3 "$OUT/pytest_gpu.log"
run 180 "$OUT/smoke.log" python -u -c "import __graft_entry__ as g; g.smoke()"
run 600 "$OUT/bench.json" python -u bench.py
cat "$OUT/bench.json" | tail -1 | cut -c1-600
