#!/bin/bash
# FedAvg at several K against another library build, alternating on one box.
#   usage: tools/k_sweep_ab.sh <out-dir> <other .so> [rounds]
set -o pipefail
OUT=$1; OTHER=$2; R=${3:-2}; mkdir -p "$OUT"
B="bench.py --no-sub --no-cpu-baseline --no-reference-gpu --no-check --steps 10 --warmup 2 --workload cfg3"
for i in $(seq 1 "$R"); do
  for kc in 16:46758048 64:11689512 64:46758048 256:15625000; do
    k=${kc%%:*}; c=${kc##*:}
    for who in other prod; do
      if [ $who = other ]; then export P2P_LIB=$OTHER; else unset P2P_LIB; fi
      timeout -k 10 240 python3 -u $B --peers $k --coords $c > "$OUT/${who}_k${k}_c${c}_$i.json" 2> "$OUT/${who}_k${k}_c${c}_$i.err" || exit 1
      python3 - "$OUT/${who}_k${k}_c${c}_$i.json" "$who" "$k" "$c" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:5s} K={sys.argv[3]:>4} coords={int(sys.argv[4]):>11,} frac={d['roofline']['frac']:.4f} kernel_ms={d['roofline']['kernel_ms']}")
PY
    done
  done
done
