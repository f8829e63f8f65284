# Round 6 r: the tile queue under churn (random K / sizes over three streams).
set -o pipefail
O=gpurun_out/r06r; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu -k "queue_random or two_streams or share_cus" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -6 $O/tests.log
echo done
