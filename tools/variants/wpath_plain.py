"""A/B variant (round 6): the split kernel's w path as before -- plain w
DMA, plain global stores (fedavg.hip st_w)."""
p = "fedavg.hip"
s = open(p).read()
old = "#define P2P_W_DMA_AUX 2\n"
assert old in s
s = s.replace(old, "#define P2P_W_DMA_AUX 0\n")
old = "#define P2P_W_STORE_AUX 16\n"
assert old in s
open(p, "w").write(s.replace(old, "#define P2P_W_STORE_AUX -1\n"))
