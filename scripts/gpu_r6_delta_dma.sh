#!/bin/bash
# Round 6 (last session): the delta's LDS-DMA scheme against the product
# layout, every layout with the device-scope (sc1) stores too
# (tools/delta_dma_lab.hip, built in-tree on the CPU).
set -o pipefail
O=gpurun_out/delta_dma
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 ./tools/delta_dma_lab 268435456 11 > $O/lab_256m.log 2>&1 || { cat $O/lab_256m.log; exit 1; }
cat $O/lab_256m.log
timeout -k 10 300 ./tools/delta_dma_lab 1073741824 7 > $O/lab_1b.log 2>&1 || { cat $O/lab_1b.log; exit 1; }
cat $O/lab_1b.log
