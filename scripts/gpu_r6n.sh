# Round 6 n: host profile of the general path with a new table per call, cfg1.
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 300 python -u tools/prof_general.py 200 mlp > $O/prof_general_mlp.log 2>&1 || { tail -30 $O/prof_general_mlp.log; exit 1; }
head -60 $O/prof_general_mlp.log
echo done
