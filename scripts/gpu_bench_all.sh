#!/bin/bash
# Every bench workload (one process each, own time limits) + a 2-rank gloo
# rehearsal of the N>1 path + rocprofv3 stats of the robust kernels.
set -u
TAG=${1:-all}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
run() { local name=$1 t=$2; shift 2; local s=$SECONDS
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc $((SECONDS-s))s"; tail -1 "$OUT/$name.log" | cut -c1-300; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench_cfg3 600 python bench.py || exit $?
run bench_cfg2 300 python bench.py --workload cfg2 --steps 50 --warmup 5 --no-cpu-baseline || exit $?
run bench_cfg1 300 python bench.py --workload cfg1 || exit $?
run bench_cfg4m 300 python bench.py --workload cfg4-median --steps 5 --warmup 1 --cpu-seconds 8 || exit $?
run bench_cfg4t 300 python bench.py --workload cfg4-trimmed --steps 5 --warmup 1 --no-cpu-baseline || exit $?
run bench_med256 300 python bench.py --workload median256 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
run bench_trim256 300 python bench.py --workload trimmed256 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
run bench_delta 300 python bench.py --workload delta --steps 10 --warmup 2 --cpu-seconds 8 || exit $?
run bench_sha 300 python bench.py --workload sha256 --coords 1000000 --steps 3 --warmup 1 --cpu-seconds 5 || exit $?
run bench_cfg5 600 python bench.py --workload cfg5 --steps 2 --warmup 1 --no-cpu-baseline || exit $?
run dist2_gloo 600 env P2P_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --coords 8388608 --peers 16 --steps 3 --warmup 1 --chunks 4 || exit $?
cd /tmp
run stats_robust 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats_robust" -o bench -- python3 "$ROOT/bench.py" --workload median256 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
