"""A/B variant (round 6): the split kernel's tile queue on (P2P_SPLIT_QUEUE 1)."""
p = "fedavg.hip"
s = open(p).read()
old = "#define P2P_SPLIT_QUEUE 0"
assert old in s
open(p, "w").write(s.replace(old, "#define P2P_SPLIT_QUEUE 1"))
