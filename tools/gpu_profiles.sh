#!/bin/bash
# One gpurun call: the profiles committed under profiles/<round>/ --
#   * rocprofv3 --kernel-trace --stats of the default bench line (every
#     record's kernel, the numbers bench.py's HIP events must agree with);
#   * HBM traffic per launch for every bench record (FETCH_SIZE and
#     WRITE_SIZE in separate passes, tools/pmc_traffic.py -> traffic_*.json);
#   * SQ / GRBM counters of the robust kernels (K = 256 and cfg4).
# Each GPU step has its own time limit; the chain stops at the first failure.
#   usage: tools/gpu_profiles.sh <out-dir under gpurun_out/>
set -o pipefail
OUT=${1:-gpurun_out/profiles}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1

run() {  # run <seconds> <log> <cmd...>
  local secs=$1 logf=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$logf" 2>&1
  local rc=$?
  echo "== rc=$rc" | tee -a "$OUT/steps.log"
  [ $rc -eq 0 ] || { tail -30 "$logf"; exit $rc; }
}
F="--output-format csv"
B="bench.py --no-sub --no-cpu-baseline --no-reference-gpu --steps 2 --warmup 1"

# ONLY="cfg3 delta ..." limits the traffic passes (and skips the SQ passes
# unless one of their workloads is named); NO_STATS=1 skips the stats run.
# kernel stats of the default bench (all sub-records), CPU baselines skipped
[ -n "$NO_STATS" ] || run 600 "$OUT/stats_bench.log" rocprofv3 --kernel-trace --stats $F -d "$OUT/stats_bench" -o bench -- python3 -u bench.py --no-cpu-baseline

# HBM traffic per launch (one launch per chunk-major plane, sharded.PeerPlanes):
# workload kernel coords-per-launch peers [extra bench args]
while IFS=: read -r w k c p extra; do
  [ -z "$w" ] && continue
  [ -n "$ONLY" ] && [[ " $ONLY " != *" $w "* ]] && continue
  for cn in FETCH_SIZE WRITE_SIZE; do
    run 240 "$OUT/pmc_${cn}_$w.log" timeout -s KILL 220 rocprofv3 --pmc $cn $F -d "$OUT/pmc_${cn}_$w" -o run -- python3 -u $B $extra
  done
  python3 tools/pmc_traffic.py "$OUT/pmc_FETCH_SIZE_$w" "$OUT/pmc_WRITE_SIZE_$w" "$k" "$w" "$c" "$p" "$OUT/traffic_$w.json" > /dev/null || exit 1
done <<'EOS'
cfg3:fedavg_split_kernel+fedavg_flat_kernel:15625000:256:--workload cfg3
cfg3-chunk:fedavg_split_kernel+fedavg_flat_kernel:15625000:256:--job cfg3-full --steps 1
cfg2-dropin:fedavg_split_kernel<false, 2,:11689512:64:--workload cfg2-dropin
cfg4-median:robust_flat_kernel:25000000:128:--workload cfg4-median
cfg4-trimmed:robust_flat_kernel:25000000:128:--workload cfg4-trimmed
median256:robust_median_pair_kernel:12500000:256:--workload median256
trimmed256:robust_pair_kernel:12500000:256:--workload trimmed256
delta:delta_flat_kernel:1000000000:1:--workload delta
EOS

# issue / wait / clock counters of the K = 256 robust kernels (8 SQ + 2 GRBM slots)
for w in median256 trimmed256 cfg4-median cfg4-trimmed; do
  [ -n "$ONLY" ] && [[ " $ONLY " != *" $w "* ]] && continue
  run 240 "$OUT/pmc_sq_$w.log" timeout -s KILL 220 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT $F -d "$OUT/pmc_sq_$w" -o run -- python3 -u $B --workload $w
  python3 tools/rocpd_summary.py "$OUT/pmc_sq_$w" robust > "$OUT/sq_$w.json" || true
done
ls "$OUT"
