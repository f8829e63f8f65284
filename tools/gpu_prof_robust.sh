#!/bin/bash
# One gpurun call: robust-rule A/B (lab library), the diag split of the
# K = 256 kernels, rocprofv3 kernel stats, SQ/GRBM PMC and HBM-traffic passes.
# Each GPU step has its own time limit; the chain stops at the first failure.
#   usage: tools/gpu_prof_robust.sh <out-dir under gpurun_out/>
set -o pipefail
OUT=${1:-gpurun_out/prof}
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
B="bench.py --no-sub --no-cpu-baseline --steps 5 --warmup 1"

# A/B of the K = 256 median variants (bit-compared with the product kernel)
run 300 "$OUT/lab_med256_uniform.log" python -u tools/lab_robust.py --rule median --peers 256 --variants 0,1
run 300 "$OUT/lab_med256_quantized.log" python -u tools/lab_robust.py --rule median --peers 256 --variants 0,1 --data quantized --coords 20000000
run 300 "$OUT/lab_med256_normal.log" python -u tools/lab_robust.py --rule median --peers 256 --variants 0,1 --data normal --coords 20000000
grep -h '^{' "$OUT"/lab_*.log

# diag split (wrong results by design; timing only)
for w in median256 trimmed256; do
  for d in 1 2 3; do
    [ "$w" = median256 ] && [ $d = 3 ] && continue
    P2P_LIB=tools/libp2pdl_diag$d.so run 200 "$OUT/diag${d}_$w.log" python -u $B --workload $w --no-check
  done
done
grep -h '"kernel_ms"' "$OUT"/diag*.log | sed 's/.*"workload": "\([^:]*\):.*"kernel_ms": \([0-9.]*\).*/\1 \2/'

# kernel stats
for w in median256 trimmed256; do
  run 300 "$OUT/stats_$w.log" rocprofv3 --kernel-trace --stats -d "$OUT/stats_$w" -o run -- python3 -u $B --workload $w
done
# SQ + GRBM counters (one pass each workload; 8 SQ + 2 GRBM slots)
for w in median256 trimmed256; do
  run 200 "$OUT/pmc_sq_$w.log" timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d "$OUT/pmc_sq_$w" -o run -- python3 -u $B --workload $w --steps 2
done
# HBM traffic (FETCH_SIZE and WRITE_SIZE in separate passes)
for spec in "trimmed256:robust_lds_kernel:100000000:256" "cfg4-trimmed:robust_flat_kernel:100000000:128" "cfg2-dropin:fedavg_segments_kernel:11689512:64"; do
  IFS=: read w k c p <<< "$spec"
  for cn in FETCH_SIZE WRITE_SIZE; do
    run 200 "$OUT/pmc_${cn}_$w.log" timeout -s KILL 180 rocprofv3 --pmc $cn -d "$OUT/pmc_${cn}_$w" -o run -- python3 -u $B --workload $w --steps 2
  done
  python3 tools/pmc_traffic.py "$OUT/pmc_FETCH_SIZE_$w" "$OUT/pmc_WRITE_SIZE_$w" "$k" "$w" "$c" "$p" "$OUT/traffic_$w.json" > /dev/null || exit 1
done
ls "$OUT"
