#!/bin/bash
# Robust-kernel diagnosis: full kernel vs no-DMA / no-sort builds + SQ counters.
set -u
TAG=${1:-diag}; WL=${2:-median256}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
run() { local name=$1 t=$2; shift 2; local s=$SECONDS
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc $((SECONDS-s))s"; tail -1 "$OUT/$name.log" | python3 -c "import sys,json
l=sys.stdin.read().strip()
try:
  j=json.loads(l); print('   ', j['config']['workload'], 'value', j['value'], 'kernel_ms', j['roofline']['kernel_ms'], 'frac', j['roofline']['frac'])
except Exception: print(l[-600:])"; return $rc; }
run full 300 python bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline || exit $?
run nodma 300 env P2P_LIB=$ROOT/p2pdl_amd/libp2pdl_hip_diag1.so python bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-check || exit $?
run nosort 300 env P2P_LIB=$ROOT/p2pdl_amd/libp2pdl_hip_diag2.so python bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-check || exit $?
cd /tmp
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"}
run pmc_sq 120 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/pmc_sq" -o bench -- python3 "$ROOT/bench.py" --workload $WL --coords 20000000 --steps 1 --warmup 1 --no-cpu-baseline --no-check || exit $?
python3 - "$OUT/pmc_sq" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    if "synth" in r["Kernel_Name"]: continue
    agg[(r["Kernel_Name"][:60], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k[0], k[1]); print("   ", {c: round(x) for c, x in sorted(v.items())})
PY
