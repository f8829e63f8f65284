set -o pipefail
O=gpurun_out/r05/t5
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "delta" tests/test_c_host.py tests/test_abi.py > $O/pytest.log 2>&1 || exit 1
for w in delta cfg1 cfg2-dropin cfg5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 2 --cpu-seconds 3 > $O/$w.json 2> $O/$w.err || exit 2
done
