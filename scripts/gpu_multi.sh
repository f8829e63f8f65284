#!/bin/bash
# Multi-rank rehearsal on ONE GPU (gloo, ranks share cuda:0) + robust benches.
set -u
TAG=${1:-multi}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
run() { local name=$1 t=$2; shift 2; local s=$SECONDS
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc $((SECONDS-s))s"; tail -3 "$OUT/$name.log" | cut -c1-700; return $rc; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -rf; rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
run dist2_gloo 600 env P2P_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --coords 8388608 --peers 16 --steps 3 --warmup 1 --chunks 4 || exit $?
run dist1_nccl 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu-baseline || exit $?
run med128 600 python bench.py --workload cfg4-median --steps 5 --warmup 1 --no-cpu-baseline || exit $?
run trim128 600 python bench.py --workload cfg4-trimmed --steps 5 --warmup 1 --no-cpu-baseline || exit $?
run med256 600 python bench.py --workload median256 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
run trim256 600 python bench.py --workload trimmed256 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
