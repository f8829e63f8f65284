#!/bin/bash
# Native parser on the box: inbox GPU tests + the inbox bench record.
set -o pipefail
OUT=${1:-gpurun_out/r4c}; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_inbox.py tests/test_inbox_ownership.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --workload inbox --steps 5 --warmup 2 > "$OUT/inbox.log" 2>&1 || { tail -20 "$OUT/inbox.log"; exit 1; }
grep -h '^{' "$OUT/inbox.log" | cut -c1-1500
timeout -k 10 300 python -u tools/inbox_split_probe.py > "$OUT/split.log" 2>&1 || { tail -20 "$OUT/split.log"; exit 1; }
tail -12 "$OUT/split.log"
