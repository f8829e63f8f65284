#!/bin/bash
# FedAvg variant sweep + PMC HBM-traffic passes for the cfg3 bench kernel.
set -u
TAG=${1:-sweep}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
run() { local name=$1 t=$2; shift 2; local s=$SECONDS
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc $((SECONDS-s))s"; tail -4 "$OUT/$name.log"; return $rc; }
run sweep_k256 300 ./tools/fedavg_sweep 256 33554432 3 || exit $?
run sweep_k64 300 ./tools/fedavg_sweep 64 11689512 5 || exit $?
cd /tmp
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o bench -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-check || exit $?
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o bench -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-check || exit $?
