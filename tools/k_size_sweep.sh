#!/bin/bash
# FedAvg efficiency against K and size on one box: the cfg3 bench line's
# flat planes at (K, coordinates) pairs of equal and growing bytes.
#   usage: tools/k_size_sweep.sh <out-dir>
set -o pipefail
OUT=$1; mkdir -p "$OUT"
B="bench.py --no-sub --no-cpu-baseline --no-reference-gpu --no-check --steps 10 --warmup 2 --workload cfg3"
for kc in 64:11689512 64:46758048 64:62500000 256:2922378 256:15625000 16:46758048; do
  k=${kc%%:*}; c=${kc##*:}
  timeout -k 10 240 python3 -u $B --peers $k --coords $c > "$OUT/k${k}_c${c}.json" 2> "$OUT/k${k}_c${c}.err" || exit 1
  python3 - "$OUT/k${k}_c${c}.json" "$k" "$c" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"K={sys.argv[2]:>4} coords={int(sys.argv[3]):>11,} frac={d['roofline']['frac']:.4f} kernel_ms={d['roofline']['kernel_ms']} layout={d['config'].get('layout')}")
PY
done
