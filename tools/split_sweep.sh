#!/bin/bash
# Size sweep of tools/fedavg_split (one process per size, each bounded).
set -o pipefail
out=${1:-gpurun_out/r05/split3}
mkdir -p "$out"
for kn in "256 16777216" "256 2097152" "256 8388608" "256 33554432" "64 33554432" "256 124993536"; do
  set -- $kn
  echo "== K=$1 n=$2" | tee -a "$out/lab.log"
  timeout -k 10 200 ./tools/fedavg_split $1 $2 5 >> "$out/lab.log" 2>&1 || { echo "FAILED rc=$? at K=$1 n=$2"; exit 1; }
done
