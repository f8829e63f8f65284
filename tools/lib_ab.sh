#!/bin/bash
# Same-box A/B of the product library against another build (P2P_LIB) on
# bench workloads, alternating processes.
#   usage: tools/lib_ab.sh <out-dir> <other .so> <rounds> <workload> [<workload> ...]
set -o pipefail
OUT=$1; OTHER=$2; R=$3; shift 3
mkdir -p "$OUT"
B="bench.py --no-sub --no-cpu-baseline --no-reference-gpu --steps 10 --warmup 2"
for i in $(seq 1 "$R"); do
  for w in "$@"; do
    P2P_LIB=$OTHER timeout -k 10 240 python3 -u $B --workload $w > "$OUT/other_${w}_$i.json" 2> "$OUT/other_${w}_$i.err" || exit 1
    timeout -k 10 240 python3 -u $B --workload $w > "$OUT/prod_${w}_$i.json" 2> "$OUT/prod_${w}_$i.err" || exit 1
  done
done
python3 - "$OUT" <<'PY'
import glob, json, os, sys
rows = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            who, w = os.path.basename(f).split("_", 1)
            rows.setdefault((w.rsplit("_", 1)[0], who), []).append(d["roofline"]["frac"])
for (w, who), v in sorted(rows.items()):
    print(f"{w:14s} {who:6s} " + " ".join(f"{x:.4f}" for x in v))
PY
