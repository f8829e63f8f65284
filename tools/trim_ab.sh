#!/bin/bash
# Same-box A/B of two builds of the library (P2P_LIB) on the robust K = 256
# records, alternating processes; then SQ counters of the new build.
#   usage: tools/trim_ab.sh <out-dir> <old .so> [rounds]
set -o pipefail
OUT=$1; OLD=$2; R=${3:-2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="bench.py --no-sub --no-cpu-baseline --no-reference-gpu --steps 8 --warmup 2"
for i in $(seq 1 "$R"); do
  for w in trimmed256 median256; do
    P2P_LIB=$OLD timeout -k 10 240 python3 -u $B --workload $w > "$OUT/old_${w}_$i.json" 2> "$OUT/old_${w}_$i.err" || exit 1
    timeout -k 10 240 python3 -u $B --workload $w > "$OUT/new_${w}_$i.json" 2> "$OUT/new_${w}_$i.err" || exit 1
  done
done
for w in trimmed256 median256; do
  timeout -s KILL 220 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmc_sq_$w" -o run -- python3 -u bench.py --no-sub --no-cpu-baseline --no-reference-gpu --steps 2 --warmup 1 --workload $w > "$OUT/pmc_sq_$w.log" 2>&1 || exit 1
  python3 tools/rocpd_summary.py "$OUT/pmc_sq_$w" robust > "$OUT/sq_$w.json" || true
done
