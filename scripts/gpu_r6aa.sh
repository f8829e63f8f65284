# Round 6 aa: the adopted split-kernel w path (nt w DMA + sc1 stores) -- the
# GPU suite, the delta's store-policy A/B, the adopted build against the
# previous plain w path, and the main line.
set -o pipefail
O=gpurun_out/r06aa; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python -u tools/lib_pair_ab.py 15 prod delta_nt delta_s16 delta_s17 delta_s18 delta_s19 -- delta:1000000000 delta:125000000 > $O/delta_ab.log 2>&1 || { tail -30 $O/delta_ab.log; exit 1; }
cat $O/delta_ab.log
timeout -k 10 400 python -u tools/lib_pair_ab.py 15 prod wpath_plain -- 256:16777216 64:100007936 rows:64:1 sd:64:1 > $O/wpath_adopted_ab.log 2>&1 || { tail -30 $O/wpath_adopted_ab.log; exit 1; }
cat $O/wpath_adopted_ab.log
timeout -k 10 300 python -u bench.py --no-sub --no-cpu-baseline > $O/main.json 2> $O/main.err || { tail -30 $O/main.err; exit 1; }
cut -c1-300 $O/main.json
