# Round 6 z: the split kernel's w path in the product library -- nontemporal
# w DMA and the epilogue's stores with cache-policy bits (tools/variants/
# wpath_*.py) against the current product, same process, launch by launch.
set -o pipefail
O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 600 python -u tools/lib_pair_ab.py 15 prod wpath_nt2 wpath_s16 wpath_s17 wpath_s18 wpath_s19 -- \
  256:16777216 64:100007936 16:11689984 16:100007936 rows:64:1 sd:64:1 > $O/wpath_ab.log 2>&1 || { tail -30 $O/wpath_ab.log; exit 1; }
cat $O/wpath_ab.log
