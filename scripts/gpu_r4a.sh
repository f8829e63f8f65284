#!/bin/bash
# Round-4 check of the ownership / digest / sharding changes, then the
# self-launching --gpus 2 rehearsal (gloo, both ranks on the one GPU).
set -o pipefail
OUT=${1:-gpurun_out/r4a}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu \
  tests/test_inbox_ownership.py tests/test_inbox.py tests/test_sharded.py tests/test_crypto.py \
  tests/test_host_tables.py > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
P2P_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 3 --warmup 1 --coords 20000000 \
  --no-cpu-baseline > "$OUT/dist2_spawn.log" 2>&1 || { tail -30 "$OUT/dist2_spawn.log"; exit 1; }
grep -h '^{' "$OUT/dist2_spawn.log" | cut -c1-900
