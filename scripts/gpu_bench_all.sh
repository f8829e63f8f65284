#!/bin/bash
# GPU parity tests + every bench workload (one process each, own time limits).
set -u
TAG=${1:-all}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
run() { local name=$1 t=$2; shift 2; local s=$SECONDS
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc $((SECONDS-s))s"; tail -2 "$OUT/$name.log" | cut -c1-1500; return $rc; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -rf; rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
run bench_cfg3 600 python bench.py --steps 10 --warmup 2 || exit $?
run bench_cfg2 300 python bench.py --workload cfg2 --steps 50 --warmup 5 --no-cpu-baseline || exit $?
run bench_cfg4m 600 python bench.py --workload cfg4-median --steps 5 --warmup 1 --cpu-seconds 8 || exit $?
run bench_cfg4t 600 python bench.py --workload cfg4-trimmed --steps 5 --warmup 1 --no-cpu-baseline || exit $?
run bench_sha 600 python bench.py --workload sha256 --coords 1000000 --steps 3 --warmup 1 --cpu-seconds 5 || exit $?
run bench_cfg5 900 python bench.py --workload cfg5 --coords 2500000 --steps 2 --warmup 1 --no-cpu-baseline || exit $?
