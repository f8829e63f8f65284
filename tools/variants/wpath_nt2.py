"""A/B variant (round 6): the split kernel's w path -- w DMA cache policy
2, epilogue stores as buffer stores with cache-policy bits 2 (bit 0
sc0, bit 1 nt, bit 4 sc1); see fedavg.hip st_w."""
p = "fedavg.hip"
s = open(p).read()
old = "#define P2P_W_DMA_AUX 2\n"
assert old in s
s = s.replace(old, "#define P2P_W_DMA_AUX 2\n")
old = "#define P2P_W_STORE_AUX 16\n"
assert old in s
open(p, "w").write(s.replace(old, "#define P2P_W_STORE_AUX 2\n"))
