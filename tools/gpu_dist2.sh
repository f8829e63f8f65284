#!/bin/bash
# World-size-2 rehearsal of the bench's multi-GPU path on ONE GPU (gloo,
# both ranks on cuda:0): the default line (cfg3 tile per rank + cfg3_full
# job) at reduced size.  The driver's real N>1 runs use RCCL, one GPU per rank.
set -o pipefail
OUT=${1:-gpurun_out/dist2}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
P2P_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 3 --warmup 1 --coords 20000000 \
  --no-cpu-baseline > "$OUT/dist2_flat.log" 2>&1 || { tail -30 "$OUT/dist2_flat.log"; exit 1; }
grep -h '^{' "$OUT/dist2_flat.log" | cut -c1-700
