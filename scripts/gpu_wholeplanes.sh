#!/bin/bash
# Round 5: whole-round planes on cfg3 -- GPU tests of sharded.py, the default
# bench line, PMC traffic and kernel stats of the cfg3 record.
set -o pipefail
O=gpurun_out/wp2
mkdir -p $O/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="python3 -u bench.py --no-sub --no-cpu-baseline --no-reference-gpu --steps 2 --warmup 1 --workload cfg3"
timeout -k 10 300 python3 -u -m pytest tests/test_sharded.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 420 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof/pmc_FETCH_SIZE_cfg3 -o run -- $B > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof/pmc_WRITE_SIZE_cfg3 -o run -- $B > $O/pmc_write.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof/stats_cfg3 -o run -- python3 -u bench.py --no-sub --no-cpu-baseline --no-reference-gpu --steps 10 --warmup 2 --workload cfg3 > $O/stats_bench.json 2> $O/stats.err
echo "rc=$?" >> $O/done.txt
