#!/bin/bash
# One gpurun call: a pytest subset and a list of bench runs, each under its own
# time limit; stops at the first failure.
#   usage: tools/gpu_quick.sh <out-dir> "<pytest -k expr or empty>" "<bench args>" ["<bench args>" ...]
set -o pipefail
OUT=$1; K=$2; shift 2
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
i=0
for b in "$@"; do
  i=$((i+1))
  timeout -k 10 400 python -u bench.py $b > "$OUT/bench$i.log" 2>&1 || { tail -30 "$OUT/bench$i.log"; exit 1; }
  echo "== bench.py $b"; grep -h '^{' "$OUT/bench$i.log" | cut -c1-1500
done
