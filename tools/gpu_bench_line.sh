set -o pipefail
mkdir -p gpurun_out/r03_bench1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench1/line.json 2> gpurun_out/r03_bench1/stderr.log
rc=$?
tail -c 600 gpurun_out/r03_bench1/line.json; echo; wc -c gpurun_out/r03_bench1/line.json
exit $rc
