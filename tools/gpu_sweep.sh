#!/bin/bash
# One gpurun call: every bench.py workload with its CPU baseline (one JSON
# line each), after the default line.  Each run has its own time limit; the
# chain stops at the first failure.
#   usage: tools/gpu_sweep.sh <out-dir under gpurun_out/> [workload ...]
set -o pipefail
OUT=${1:-gpurun_out/sweep}; shift
WL=${*:-cfg1 cfg2 sha256 cfg5 delta inbox}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for w in $WL; do
  echo "== $(date +%T) $w" | tee -a "$OUT/steps.log"
  timeout -k 10 400 python -u bench.py --workload $w --no-sub > "$OUT/bench_$w.log" 2>&1
  rc=$?; echo "== rc=$rc" | tee -a "$OUT/steps.log"
  [ $rc -eq 0 ] || { tail -30 "$OUT/bench_$w.log"; exit $rc; }
  grep -h '^{' "$OUT/bench_$w.log" | cut -c1-900
done
