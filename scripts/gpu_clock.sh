#!/bin/bash
# Effective shader clock (GRBM_GUI_ACTIVE / 8 / duration) of a bench kernel,
# product vs diagnostic builds.
set -u
TAG=${1:-clock}; WL=${2:-median256}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for lib in product ${LIBS:-diag1 diag2}; do
  if [ $lib = product ]; then envs=""; else envs="P2P_LIB=$ROOT/p2pdl_amd/libp2pdl_hip_$lib.so"; fi
  env $envs timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/$lib" -o bench -- python3 "$ROOT/bench.py" --workload $WL --coords ${COORDS:-40000000} --steps 2 --warmup 1 --no-cpu-baseline --no-check > "$OUT/$lib.log" 2>&1 || { echo "$lib failed"; tail -5 "$OUT/$lib.log"; exit 1; }
  python3 - "$OUT/$lib" $lib <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); dur = {}
for r in csv.DictReader(open(f)):
    if "synth" in r["Kernel_Name"] or "copyBuffer" in r["Kernel_Name"]: continue
    key = (r["Kernel_Name"][:50], r["Dispatch_Id"])
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
for k, v in agg.items():
    d = dur[k]
    print(sys.argv[2], k[0], "dur_ms %.3f" % (d * 1e3), "clk_GHz %.3f" % (v["GRBM_GUI_ACTIVE"] / 8 / d / 1e9),
          "valu/wavecyc %.3f" % (v["SQ_INSTS_VALU"] / max(v["SQ_WAVE_CYCLES"], 1)),
          "wait_inst %.2f active %.2f" % (v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"], v["SQ_ACTIVE_INST_ANY"] / v["SQ_WAVE_CYCLES"]))
PY
done
