#!/bin/bash
# Round 6 (last session): the gloo N = 2 rehearsal of bench's multi-GPU line
# on the final tree (both ranks on the one GPU), all three exchange legs.
set -o pipefail
bash tools/gpu_dist2.sh gpurun_out/dist2_final || exit $?
echo done
