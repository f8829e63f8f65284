"""A/B variant (round 6): the tile queue's early claim schedule (claim at a
tile's start) and the queue only up to K = 128 -- the product before the
late schedule."""
p = "fedavg.hip"
s = open(p).read()
for old, new in (("#define P2P_QUEUE_LATE 1", "#define P2P_QUEUE_LATE 0"),
                 ("constexpr int kQueueMaxK = 256;", "constexpr int kQueueMaxK = 128;")):
    assert old in s
    s = s.replace(old, new)
open(p, "w").write(s)
