# Round 6 g: same-process A/B (tools/lib_pair_ab.py, builds alternated rep by
# rep) of the product (queue + every whole tile) against no queue (round 5's
# plan) and queue + whole rounds, on flat FedAvg shapes.
set -o pipefail
O=gpurun_out/r06g; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u tools/lib_pair_ab.py 20 prod noqueue qrounds -- 256:16777216 256:7559488 256:15625000 \
  64:100007936 16:100007936 64:11689984 16:11689984 sd:64:1 sd:16:1 sd:64:4 > $O/pair_ab.log 2>&1 || { tail -30 $O/pair_ab.log; exit 1; }
cat $O/pair_ab.log
echo done
