# Round 6 ab: the robust kernels' store policy (tools/variants/robust_*.py)
# against the product, same process, launch by launch.
set -o pipefail
O=gpurun_out/r06ab; mkdir -p $O
timeout -k 10 600 python -u tools/lib_pair_ab.py 11 prod robust_nt robust_s16 robust_s18 -- \
  256:12500000:median 256:12500000:trimmed 128:50000000:median 128:50000000:trimmed > $O/robust_ab.log 2>&1 || { tail -30 $O/robust_ab.log; exit 1; }
cat $O/robust_ab.log
