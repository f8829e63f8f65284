#!/bin/bash
# Round 6 (last session): does the caching allocator's configuration change
# the clones' translation cost?  The bench's cfg2 setup (rowsclone) under the
# default allocator and under expandable segments, plus its UTCL1 misses.
set -o pipefail
O=gpurun_out/alloc_conf
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u tools/lib_pair_ab.py 30 prod -- rowsclone:64:1 rowsclone:16:1 > $O/default.log 2>&1 || { tail -20 $O/default.log; exit 1; }
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 300 python3 -u tools/lib_pair_ab.py 30 prod -- rowsclone:64:1 rowsclone:16:1 > $O/expandable.log 2>&1 || { tail -20 $O/expandable.log; exit 1; }
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_SERIALIZATION_STALL_sum --output-format csv -d $O/p1 -o run -- python3 -u tools/lib_pair_ab.py 6 prod -- rowsclone:64:1 > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
python3 tools/tlb_summary.py $O/p1 $O/tlb_expandable.json > /dev/null
grep -v amdgpu.ids $O/default.log; echo "--- expandable_segments"; grep -v amdgpu.ids $O/expandable.log
python3 -c "import json;d=json.load(open('$O/tlb_expandable.json'));print({k:round(v['TCP_UTCL1_TRANSLATION_MISS_sum']) for k,v in d.items()})"
