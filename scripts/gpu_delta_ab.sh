#!/bin/bash
# A/B of the trainer-delta flat kernel knobs (P2P_DELTA_NV x P2P_DELTA_NT).
set -u
TAG=${1:-delta_ab}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for PS in ${PSS:-0}; do for NT in ${NTS:-1 0}; do for NV in ${NVS:-1 2 4 8}; do
  timeout -k 10 200 env P2P_DELTA_NV=$NV P2P_DELTA_NT=$NT P2P_DELTA_PERSIST=$PS python bench.py --workload delta --steps 20 --warmup 3 \
    --no-cpu-baseline > "$OUT/nv${NV}_nt${NT}_p${PS}.log" 2>&1 || { echo "nv$NV nt$NT failed rc=$?"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],3),'ms', round(r['achieved']), 'GB/s', round(r['frac'],4))" "$OUT/nv${NV}_nt${NT}_p${PS}.log" "nv$NV nt$NT p$PS"
done; done; done
# Reference points on the same box: torch's own copy_ (1 read + 1 write stream)
# and sub (2 reads + 1 write), same 1B fp32 elements.
timeout -k 10 200 python - <<'PY'
import torch
n = 1_000_000_000
a = torch.empty(n, device="cuda").uniform_(); b = torch.empty_like(a); c = torch.empty_like(a)
def t(fn, nbytes, name, reps=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"{name}: {ms:.3f} ms {nbytes/ms/1e6:.0f} GB/s {nbytes/ms/1e6/8000:.4f}")
t(lambda: b.copy_(a), 8 * n, "torch copy_")
t(lambda: torch.sub(a, b, out=c), 12 * n, "torch sub")
PY
