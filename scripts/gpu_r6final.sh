# Round 6: the one validation pass (GPU suite, smoke, default line) and the
# profiles of the same tree (rocprofv3 kernel stats of the default line, PMC
# HBM traffic of the FedAvg records whose kernels changed this round).
set -o pipefail
bash tools/final_pass.sh gpurun_out/r06final || exit 1
tail -2 gpurun_out/r06final/pytest_gpu.log
tail -1 gpurun_out/r06final/smoke.log
cut -c1-600 gpurun_out/r06final/bench.json
ONLY="cfg3 cfg3-chunk cfg2-dropin" bash tools/gpu_profiles.sh gpurun_out/r06final/prof || exit 1
echo done
