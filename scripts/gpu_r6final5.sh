# Round 6: the validation pass of the final tree (table fields as scalar loads, reserved queue pairs for captured launches)
# -- GPU suite, smoke, default line -- and its profiles: rocprofv3 kernel
# stats of the main line alone and of the whole default line, PMC HBM traffic
# of the FedAvg records.
set -o pipefail
bash tools/final_pass.sh gpurun_out/r06final5 || exit 1
tail -2 gpurun_out/r06final5/pytest_gpu.log
tail -1 gpurun_out/r06final5/smoke.log
cut -c1-400 gpurun_out/r06final5/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06final5/stats_main -o main -- python3 -u bench.py --no-sub --no-cpu-baseline --no-reference-gpu --steps 10 > gpurun_out/r06final5/stats_main.log 2>&1 || { tail -30 gpurun_out/r06final5/stats_main.log; exit 1; }
ONLY="cfg3 cfg3-chunk cfg2-dropin" bash tools/gpu_profiles.sh gpurun_out/r06final5/prof || exit 1
echo done
