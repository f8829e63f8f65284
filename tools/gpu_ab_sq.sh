#!/bin/bash
# One gpurun call: the robust GPU tests, an interleaved same-box A/B of the
# product library against an alternative build, then one SQ/GRBM counter pass
# per workload on the product library.  Each GPU step has its own time limit;
# the chain stops at the first failure.
#   usage: tools/gpu_ab_sq.sh <out-dir under gpurun_out/> <alt .so[:alt2.so...]> "<pytest -k expr>" [workloads...]
set -o pipefail
OUT=${1:-gpurun_out/ab}; ALT=$2; K=$3; shift 3
WL=${*:-median256 cfg4-median}
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
if [ -n "$K" ]; then
  run 900 "$OUT/pytest.log" python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K"
  tail -1 "$OUT/pytest.log"
fi
B="bench.py --no-sub --no-cpu-baseline --steps 10 --warmup 2"
for w in $WL; do
  for rep in 1 2; do
    run 300 "$OUT/prod${rep}_$w.log" python -u $B --workload $w
    for a in ${ALT//:/ }; do
      P2P_LIB=$a run 300 "$OUT/$(basename $a .so)_${rep}_$w.log" python -u $B --workload $w
    done
  done
done
for f in "$OUT"/prod*.log "$OUT"/lib*.log; do
  [ -f "$f" ] && echo "$(basename $f .log) $(grep -h '"kernel_ms"' $f | sed 's/.*"frac": \([0-9.]*\).*"kernel_ms": \([0-9.]*\).*/frac=\1 kernel_ms=\2/')"
done
# counters with the kernel trace (durations -> effective clock), for the
# product library and every alternative
PMC="--kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
for w in $WL; do
  run 200 "$OUT/pmc_sq_$w.log" timeout -s KILL 180 rocprofv3 $PMC -d "$OUT/pmc_sq_$w" -o run -- python3 -u $B --workload $w --steps 2
  python3 tools/rocpd_summary.py "$OUT/pmc_sq_$w" robust > "$OUT/sq_$w.json" || true
  for a in ${ALT//:/ }; do
    P2P_LIB=$a run 200 "$OUT/pmc_sq_$(basename $a .so)_$w.log" timeout -s KILL 180 rocprofv3 $PMC -d "$OUT/pmc_sq_$(basename $a .so)_$w" -o run -- python3 -u $B --workload $w --steps 2
    python3 tools/rocpd_summary.py "$OUT/pmc_sq_$(basename $a .so)_$w" robust > "$OUT/sq_$(basename $a .so)_$w.json" || true
  done
done
python3 - "$OUT" <<'PY' || true
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "sq_*.json"))):
    d = json.load(open(f))
    for p in d.get("pmc", []):
        print(os.path.basename(f), "valu/wave=%.1f" % p.get("valu_insts_per_wave", 0), "clock=%.3f GHz" % p.get("effective_clock_ghz", 0),
              "kernel_us=%.1f" % (([k["avg_ns"] for k in d["kernels"] if k["name"] == p["kernel"]] or [0])[0] / 1e3))
PY
ls "$OUT"
