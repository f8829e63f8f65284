"""A/B variant (round 6): the trainer delta's whole-tile stores as buffer
stores with cache-policy bits 17 (bit 0 sc0, bit 1 nt, bit 4 sc1); see
delta.hip st4_tile."""
p = "delta.hip"
s = open(p).read()
old = "#define P2P_DELTA_STORE_AUX -1\n"
assert old in s
open(p, "w").write(s.replace(old, "#define P2P_DELTA_STORE_AUX 17\n"))
