#!/bin/bash
# Round 6 (last session): contiguous tile runs per CU (tools/variants/contig.py,
# translation reuse across a CU's adjacent tiles) against the product's tile
# queue and against no queue, same process: the bench's cfg2 setup
# (rowsclone) at K = 64 / 16, then a flat cfg3 plane and 64 x 100M.
set -o pipefail
O=gpurun_out/contig
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 500 python3 -u tools/lib_pair_ab.py 20 prod contig noqueue -- rowsclone:64:1 rowsclone:16:1 \
  256:16777216 64:100007936 > $O/ab.log 2>&1
rc=$?
grep -v amdgpu.ids $O/ab.log
exit $rc
