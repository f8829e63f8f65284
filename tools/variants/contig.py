"""A/B variant (round 6, last session): the split kernel without its tile
queue, on a persistent grid of min(tiles, CUs) blocks where block b takes the
CONTIGUOUS run of tiles [b R, (b + 1) R), R = ceil(tiles / G): a CU's next
tile is the adjacent 32 KiB of every peer, so its translations (one fragment
per peer) can be reused -- the UTCL1 miss-per-stage of separately allocated
tensors (profiles/r06/tlb) -- at the price of a static schedule."""
p = "fedavg.hip"
s = open(p).read()


def sub(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new)


sub("#define P2P_SPLIT_QUEUE 1", "#define P2P_SPLIT_QUEUE 0")
sub("    int64_t N = QUEUE ? K : (ntiles - b + G - 1) / G * K;\n    int64_t ti = b, tnext = ntiles, issued = 0;",
    "    const int64_t R = (ntiles + G - 1) / G, t0 = b * R, t1 = t0 + R < ntiles ? t0 + R : ntiles;\n"
    "    int64_t N = QUEUE ? K : (t1 > t0 ? (t1 - t0) * K : 0);\n"
    "    int64_t ti = QUEUE ? b : t0, tnext = ntiles, issued = 0;")
sub("        if (issued > 0) ti = QUEUE ? tnext : ti + G;", "        if (issued > 0) ti = QUEUE ? tnext : ti + 1;")
sub("    for (int64_t t = b; t < ntiles; t += G) tile(t, [](int) {});\n    return;",
    "    const int64_t R = (ntiles + G - 1) / G, t0 = b * R, t1 = t0 + R < ntiles ? t0 + R : ntiles;\n"
    "    for (int64_t t = t0; t < t1; ++t) tile(t, [](int) {});\n    return;")
sub("  const dim3 grid = split_grid(ntiles);\n  if (recip)",
    "  const dim3 grid(static_cast<unsigned>(ntiles < device_cus() ? ntiles : device_cus()));\n  if (recip)")
open(p, "w").write(s)
