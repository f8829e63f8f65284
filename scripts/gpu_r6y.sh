# Round 6 y: the split kernel's w path, part by part (lab queue kernel: nt stores, nt w DMA, no stores, no w DMA, neither)
# w path?  The lab's queue kernel (Q) against the same kernel reading the
# peers only (QR: no w DMA, no store), interleaved, at K = 256 / 64 / 16.
set -o pipefail
O=gpurun_out/r06y3; mkdir -p $O
for c in "256 16777216" "64 100007936" "16 100007936" "64 11689984"; do
  ONLY="P Q QN QNN QW QR QB0 QB2 QB3 QB16 QB17 QB18 QB19" timeout -k 10 240 tools/split_fixed_lab $c 11 >> $O/ro_lab.log 2>&1 || { tail -20 $O/ro_lab.log; exit 1; }
done
cat $O/ro_lab.log
