#!/bin/bash
# Round 6 (last session): the bench's cfg2 setup in one process -- the rows
# kernel over the slab against the chunk list over .clone()d dicts and over
# the slab's own views, alternated rep by rep (fresh and carved clones).
set -o pipefail
O=gpurun_out/rowsclone
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u tools/lib_pair_ab.py 40 prod -- rowsclone:64:1 rowsclone:64:1:carve rowsclone:16:1 > $O/ab.log 2>&1
rc=$?
grep -v amdgpu.ids $O/ab.log
exit $rc
