set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "chunk or split_segments or dropin_cfg2 or plain_dicts or abi" > gpurun_out/r06a/tests.log 2>&1 || { tail -40 gpurun_out/r06a/tests.log; exit 1; }
tail -3 gpurun_out/r06a/tests.log
timeout -k 10 300 python -u tools/chunks_ab.py 15 64:1 16:1 64:4 > gpurun_out/r06a/chunks_ab.log 2>&1 || { tail -30 gpurun_out/r06a/chunks_ab.log; exit 1; }
cat gpurun_out/r06a/chunks_ab.log
