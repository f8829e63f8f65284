#!/bin/bash
# Round 6 (last session): the GPU suite and smoke on the final tree (the
# queue's launch counter made 64-bit, a host-only change after profiles/r06/final).
set -o pipefail
O=gpurun_out/last_tests
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
