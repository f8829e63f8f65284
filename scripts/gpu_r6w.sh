# Round 6 w: balanced chunk lists (whole CU rounds) vs the product's partial last round
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O
timeout -k 10 300 python -u tools/balance_ab.py 31 > $O/balance_ab.log 2>&1 || { tail -20 $O/balance_ab.log; exit 1; }
cat $O/balance_ab.log
