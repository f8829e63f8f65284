#!/bin/bash
# Round 6: the product library against another build
# (OTHER, default noqueue: tools/libp2pdl_noqueue.so from
# tools/variants/noqueue.py, the split kernel without its tile queue),
# alternating processes on one box, on bench shapes: "<name>|<bench args>".
# (The round's first A/Bs ran the queue as the variant: "queue" vs "prod".)
#   usage: [OTHER=tag] tools/queue_ab.sh <out-dir> <rounds> "<name>|<args>" ...
set -o pipefail
OUT=$1; R=$2; shift 2
mkdir -p "$OUT"
B="bench.py --no-sub --no-cpu-baseline --no-reference-gpu --steps 10 --warmup 2"
for i in $(seq 1 "$R"); do
  for spec in "$@"; do
    name=${spec%%|*}; args=${spec#*|}
    # ABBA: the first process of a pair read 2-3% faster on these boxes,
    # whichever build it was (profiles/r06/queue_ab/README.md)
    if [ $((i % 2)) = 1 ]; then order="${OTHER:-noqueue} prod"; else order="prod ${OTHER:-noqueue}"; fi
    for lib in $order; do
      if [ $lib = prod ]; then L=""; else L="P2P_LIB=tools/libp2pdl_$lib.so"; fi
      env $L timeout -k 10 240 python3 -u $B $args > "$OUT/${lib}_${name}_$i.json" 2> "$OUT/${lib}_${name}_$i.err" \
        || { tail "$OUT/${lib}_${name}_$i.err"; exit 1; }
    done
  done
done
python3 - "$OUT" <<'PY'
import glob, json, os, sys
rows = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            who, rest = os.path.basename(f)[:-5].split("_", 1)
            name = rest.rsplit("_", 1)[0]
            r = d["roofline"]
            rows.setdefault((name, who), []).append((r["frac"], r.get("kernel_ms")))
            for s, rec in (d.get("sub") or {}).items():  # e.g. cfg3_full
                if rec.get("frac") is not None:
                    rows.setdefault((f"{name}.{s}", who), []).append((rec["frac"], rec.get("kernel_ms")))
            gp = d.get("general_path") or (d.get("config") or {}).get("general_path")
            if gp:
                rows.setdefault((name + ".general", who), []).append((gp["frac_of_hbm_peak"], gp["kernel_ms"]))
for (name, who), v in sorted(rows.items()):
    print(f"{name:14s} {who:6s} " + "  ".join(f"{f:.4f} ({k} ms)" for f, k in v))
PY
