#!/bin/bash
# rocprof stats + PMC HBM traffic for the robust (median256, cfg4-median) and delta bench kernels.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
SKIP_TESTS=1 bash scripts/gpu_profile.sh r01_pmc_med256 median256 robust_lds_kernel 100000000 256 --steps 3 || exit $?
SKIP_TESTS=1 bash scripts/gpu_profile.sh r01_pmc_cfg4m cfg4-median robust_flat_kernel 100000000 128 || exit $?
SKIP_TESTS=1 bash scripts/gpu_profile.sh r01_pmc_delta delta delta_flat_kernel 1000000000 1 || exit $?
