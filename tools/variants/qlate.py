"""A/B variant (round 6): the tile queue's late claim schedule (claim after
barrier K - 8, publish after K - 5) and the queue up to K = 256."""
p = "fedavg.hip"
s = open(p).read()
for old, new in (("#define P2P_QUEUE_LATE 0", "#define P2P_QUEUE_LATE 1"),
                 ("constexpr int kQueueMaxK = 128;", "constexpr int kQueueMaxK = 256;")):
    assert old in s
    s = s.replace(old, new)
open(p, "w").write(s)
