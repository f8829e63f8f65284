#!/bin/bash
# Round 6 (last session): the clones' translation gap against K (rowsclone
# at K = 16 / 32 / 64 / 128 / 256, the product build).
set -o pipefail
O=gpurun_out/kgap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u tools/lib_pair_ab.py 16 prod -- rowsclone:16:1 rowsclone:32:1 rowsclone:64:1 \
  rowsclone:128:1 rowsclone:256:1 > $O/ab.log 2>&1
rc=$?
grep -v amdgpu.ids $O/ab.log
exit $rc
