"""A/B variant (round 6): the tile queue up to K = 256 (the product stops at
kQueueMaxK = 128)."""
p = "fedavg.hip"
s = open(p).read()
old = "constexpr int kQueueMaxK = 128;"
assert old in s
open(p, "w").write(s.replace(old, "constexpr int kQueueMaxK = 256;"))
