#!/bin/bash
# The round's one validation pass: the GPU suite, smoke(), the default bench
# line -- each step under its own limit, stopping at the first failure.
#   usage: tools/final_pass.sh <out-dir under gpurun_out/>
set -o pipefail
OUT=${1:-gpurun_out/final}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
step() {  # step <seconds> <log> <cmd...>
  local secs=$1 logf=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$logf" 2> "$logf.err"
  local rc=$?
  echo "== rc=$rc" | tee -a "$OUT/steps.log"
  [ $rc -eq 0 ] || { tail -30 "$logf" "$logf.err"; exit $rc; }
}
step 700 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step 300 "$OUT/smoke.log" python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step 600 "$OUT/bench.json" python -u bench.py
