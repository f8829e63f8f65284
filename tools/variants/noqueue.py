"""A/B variant (round 6): the split kernel without its tile queue (one block per tile)."""
p = "fedavg.hip"
s = open(p).read()
old = "#define P2P_SPLIT_QUEUE 1"
assert old in s
open(p, "w").write(s.replace(old, "#define P2P_SPLIT_QUEUE 0"))
