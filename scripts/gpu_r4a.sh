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
mkdir -p "$OUT/prof"
timeout -k 10 300 python -u tools/prof_cfg1.py > "$OUT/prof_cfg1.log" 2>&1 || { tail -20 "$OUT/prof_cfg1.log"; exit 1; }
head -45 "$OUT/prof_cfg1.log"
timeout -k 10 300 python -u tools/digest_boundary.py "$OUT/digest_boundary.json" > "$OUT/digest_boundary.log" 2>&1 || { tail -20 "$OUT/digest_boundary.log"; exit 1; }
tail -2 "$OUT/digest_boundary.log"
timeout -k 10 300 python -u bench.py --workload cfg1 --steps 200 --warmup 5 > "$OUT/cfg1.log" 2>&1 || { tail -20 "$OUT/cfg1.log"; exit 1; }
timeout -k 10 300 python -u bench.py --workload digest-flow --steps 5 --warmup 1 > "$OUT/digest_flow.log" 2>&1 || { tail -20 "$OUT/digest_flow.log"; exit 1; }
grep -h '^{' "$OUT/cfg1.log" "$OUT/digest_flow.log" | cut -c1-1200
