# Round 6 q: the gloo N = 2 rehearsal on the final tree (share hint in the
# overlap leg, the late-claim queue in the inline leg).
set -o pipefail
O=gpurun_out/r06q; mkdir -p $O
export PYTHONUNBUFFERED=1
P2P_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --coords 20000000 \
  --no-cpu-baseline > $O/dist2.log 2>&1 || { tail -30 $O/dist2.log; exit 1; }
grep -h '^{' $O/dist2.log > $O/dist2.json
grep -h "spot check" $O/dist2.log | head
cut -c1-600 $O/dist2.json
echo done
