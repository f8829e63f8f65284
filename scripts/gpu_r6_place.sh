#!/bin/bash
# Round 6 (late): does where pickle.loads-style tensors sit change the chunk
# list's rate?  One process: one allocation per tensor, packed peer-major
# (512 B / 4 KiB rounding, the caching allocator carving a freed block), and
# one allocation per tensor viewed 512 B in; the slab rows beside them.
set -o pipefail
O=gpurun_out/place
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u tools/lib_pair_ab.py 30 prod -- sd:64:1:alloc sd:64:1:packed512 sd:64:1:packed4096 \
  sd:64:1:off512 sd:64:1:packed65536 rows:64:1 sd:16:1:alloc sd:16:1:packed512 > $O/ab.log 2>&1
rc=$?
grep -v amdgpu.ids $O/ab.log
exit $rc
