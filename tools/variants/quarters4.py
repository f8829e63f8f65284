"""A/B variant (round 6): a flat buffer's VGPR rest runs 1024-float quarter
tiles below FOUR 4096-float tiles per CU (the product: below one), e.g. the
cfg3 short plane's 154-tile rest (308 tiles of 4096 -> 1232 quarter blocks)."""
p = "fedavg.hip"
s = open(p).read()
old = "  if (P2P_FLAT_QUARTERS && ceil_div(n - done, kTile) < device_cus()) {"
assert old in s
open(p, "w").write(s.replace(old, "  if (P2P_FLAT_QUARTERS && ceil_div(n - done, kTile) < 4 * device_cus()) {"))
