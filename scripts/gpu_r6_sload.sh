#!/bin/bash
# Round 6 (late): host-built table reads as scalar loads (ldc) -- the GPU
# tests on the new build, then a same-process A/B against HEAD's build
# (tools/libp2pdl_old.so): chunk-list state_dicts, slab rows, flat control.
set -o pipefail
O=gpurun_out/sload
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
tail -2 $O/pytest.log &&
timeout -k 10 400 python3 -u tools/lib_pair_ab.py 30 prod old -- sd:64:1 sd:16:1 sd:64:4 rows:64:1 rows:16:1 256:16777216 delta:125000000 > $O/ab.log 2>&1
rc=$?
echo "rc=$rc" >> $O/done.txt
cat $O/ab.log | grep -v amdgpu.ids
exit $rc
