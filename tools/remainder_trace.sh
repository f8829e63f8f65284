#!/bin/bash
# Kernel trace of the cfg3 bench line under two library builds, alternating:
# the split kernel and its VGPR remainder per plane launch (trace_summary.py).
#   usage: tools/remainder_trace.sh <out-dir> <other .so> [rounds]
set -o pipefail
OUT=$1; OTHER=$2; R=${3:-2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="bench.py --no-sub --no-cpu-baseline --no-reference-gpu --workload cfg3 --steps 5 --warmup 1"
for i in $(seq 1 "$R"); do
  for who in other prod; do
    if [ $who = other ]; then export P2P_LIB=$OTHER; else unset P2P_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/${who}_$i" -o run -- python3 -u $B > "$OUT/${who}_$i.log" 2>&1 || exit 1
    mkdir -p "$OUT/${who}_$i/sum" && python3 tools/trace_summary.py "$OUT/${who}_$i" "$OUT/${who}_$i/sum" > /dev/null || exit 1
    python3 - "$OUT/${who}_$i/sum/kernel_trace_by_grid.json" "$who $i" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], {k.split("p2p::")[1]: v for k, v in d.items() if "fedavg" in k})
PY
  done
done
