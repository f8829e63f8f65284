#!/bin/bash
# FedAvg HBM rate vs peer-row pitch (tools/fedavg_sweep.hip), K = 256.
set -o pipefail
OUT=${1:-gpurun_out/pitch}; mkdir -p "$OUT"
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o /tmp/fs tools/fedavg_sweep.hip > "$OUT/build.log" 2>&1 || exit 1
for args in "125000000 125000000" "125000000 125829120" "125000000 134217728" "125000000 125001728" "125000000 -1" \
            "33554432 33554432" "33554432 33554496" "33554432 34603008" "100000000 100000000" "100000000 100663296"; do
  set -- $args
  timeout -k 10 120 /tmp/fs 256 $1 2 $2 1 > "$OUT/run_$1_$2.log" 2>&1 || { cat "$OUT/run_$1_$2.log"; exit 1; }
  echo "n=$1 pitch=$2"; grep -h "onetile" "$OUT/run_$1_$2.log"
done
