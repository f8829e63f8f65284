"""A/B variant (round 6): with the tile queue balancing a launch's tiles
dynamically, the split kernel takes EVERY whole tile of a flat buffer from
one CU round up (not whole rounds only); the VGPR kernel keeps the < 8192-
float tail."""
p = "fedavg.hip"
s = open(p).read()
old = "  return full / cus * cus;"
assert old in s
open(p, "w").write(s.replace(old, "  return full >= cus ? full : 0;"))
