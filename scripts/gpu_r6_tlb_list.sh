#!/bin/bash
# Round 6 (last session): which translation (UTCL) counters rocprofv3 offers on gfx950.
set -o pipefail
O=gpurun_out/tlb
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 120 rocprofv3 --list-avail > $O/list_avail.log 2>&1
rc=$?
grep -i -E "utcl|tlb|translation" $O/list_avail.log | head -60
exit $rc
