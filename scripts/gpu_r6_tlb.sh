#!/bin/bash
# Round 6 (last session): UTCL1 translation counters of the rows kernel over
# the slab and the chunk list over .clone()d dicts / the slab's views (the
# cfg2 general-path gap).  Two PMC passes of <= 4 TCP counters.
set -o pipefail
O=gpurun_out/tlb
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
P="python3 -u tools/lib_pair_ab.py 6 prod -- rowsclone:64:1"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_SERIALIZATION_STALL_sum --output-format csv -d $O/p1 -o run -- $P > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_LFIFO_FULL_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum --output-format csv -d $O/p2 -o run -- $P > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
python3 tools/tlb_summary.py $O/p1 $O/tlb_p1.json && python3 tools/tlb_summary.py $O/p2 $O/tlb_p2.json
grep -v amdgpu.ids $O/p1.log | tail -5
