#!/bin/bash
# Round 5: whole-round planes in the cfg3 full job -- N = 1 measurement, PMC
# traffic per plane launch, then the N = 2 gloo rehearsal (ranks share the GPU).
set -o pipefail
O=gpurun_out/wp4
mkdir -p $O/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="python3 -u bench.py --no-sub --no-cpu-baseline --no-reference-gpu --warmup 1 --job cfg3-full --steps 1"
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-reference-gpu --job cfg3-full --steps 2 > $O/full_n1.json 2> $O/full_n1.err &&
timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof/pmc_FETCH_SIZE_cfg3-chunk -o run -- $B > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof/pmc_WRITE_SIZE_cfg3-chunk -o run -- $B > $O/pmc_write.log 2>&1 &&
P2P_DIST_BACKEND=gloo timeout -k 10 500 python3 -u bench.py --gpus 2 --job cfg3-full --steps 1 --no-cpu-baseline --no-reference-gpu > $O/full_dist2.json 2> $O/full_dist2.err
echo "rc=$?" >> $O/done.txt
