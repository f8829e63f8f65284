#!/bin/bash
# Round 6 (late): host cost of the general path's new-table call, profiled
# call by call with a sync after each (tools/prof_general.py synced).
set -o pipefail
O=gpurun_out/host
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u tools/prof_general.py 200 synced > $O/prof_new_synced.log 2>&1 &&
timeout -k 10 300 python3 -u tools/prof_general.py 200 cached synced > $O/prof_cached_synced.log 2>&1
rc=$?
head -45 $O/prof_new_synced.log
exit $rc
