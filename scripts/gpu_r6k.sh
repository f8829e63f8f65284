# Round 6 k: the chunk kernel against the rows kernel on the same slab memory;
# rocprofv3 kernel stats of the main line alone (cfg3 planes), to set beside
# bench's own HIP-event kernel time.
set -o pipefail
O=gpurun_out/r06k; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/chunks_ab.py 20 64:1 16:1 > $O/chunks_ab.log 2>&1 || { tail -30 $O/chunks_ab.log; exit 1; }
cat $O/chunks_ab.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_main -o main -- python3 -u bench.py --no-sub --no-cpu-baseline --no-reference-gpu --steps 10 > $O/stats_main.log 2>&1 || { tail -30 $O/stats_main.log; exit 1; }
grep -h '^{' $O/stats_main.log | cut -c1-300
echo done
