#!/bin/bash
# Round 6 (last session): chunk-list loaders touching the page of the stage
# 2 / 4 ahead with a scalar load (tools/variants/xlat_pf.py) against the
# product, same process: the bench's cfg2 setup (rowsclone) at K = 64 / 16.
set -o pipefail
O=gpurun_out/xpf
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 500 python3 -u tools/lib_pair_ab.py 24 prod xpf2 xpf4 -- rowsclone:64:1 rowsclone:16:1 rowsclone:64:2 > $O/ab.log 2>&1
rc=$?
grep -v amdgpu.ids $O/ab.log
exit $rc
