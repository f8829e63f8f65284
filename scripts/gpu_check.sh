#!/bin/bash
# One GPU session: parity tests -> smoke -> benches -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; anything beyond a plain test failure
# (fault, abort, timeout) ends the script.
set -u
TAG=${1:-run}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
run() { local name=$1 t=$2; shift 2; local s=$SECONDS
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc $((SECONDS-s))s"; tail -3 "$OUT/$name.log"; return $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread; rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
for extra in "${@:2}"; do :; done
run bench_cfg2 300 python bench.py --workload cfg2 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
run bench 600 python bench.py --steps 10 --warmup 2 || exit $?
cd /tmp && run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline || exit $?
