# Round 6 m: CU sharing between the split kernel and a collective-shaped
# kernel on a second stream (tools/cu_share_lab.hip), with and without the
# share hint.
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O
for c in "64 100007936" "16 100007936" "256 16777216"; do
  set -- $c
  timeout -k 10 120 tools/cu_share_lab $1 $2 469762048 32 7 > $O/K$1.log 2>&1 || { tail $O/K$1.log; exit 1; }
  cat $O/K$1.log
done
echo done
