# Round 6 j: host profile of the general path with a new table every call;
# parity of the rows kernel on the queue (rows / drop-in tests).
set -o pipefail
O=gpurun_out/r06j; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_inbox.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "rows or dropin or inbox" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/prof_general.py 30 > $O/prof_general.log 2>&1 || { tail -30 $O/prof_general.log; exit 1; }
head -45 $O/prof_general.log
echo done
