"""A/B variant (round 6): the tile queue for the rows kernel too (the
product keeps one block per tile there)."""
p = "fedavg.hip"
s = open(p).read()
old = "  return P2P_SPLIT_QUEUE && MODE != kRows;"
assert old in s
open(p, "w").write(s.replace(old, "  return P2P_SPLIT_QUEUE;"))
