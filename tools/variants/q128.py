"""A/B variant (round 6): the late-claim tile queue only up to K = 128 (one
block per tile for the K = 256 cfg3 planes)."""
p = "fedavg.hip"
s = open(p).read()
old = "constexpr int kQueueMaxK = 256;"
assert old in s
open(p, "w").write(s.replace(old, "constexpr int kQueueMaxK = 128;"))
