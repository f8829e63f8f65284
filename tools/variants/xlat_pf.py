"""A/B variant (round 6, last session): chunk-list loaders touch the page of
the stage P ahead with one 4-byte scalar (constant address space) load of
peer data, so its translation is in the shared UTCL2 before the stage's
DMAs need it -- the clones' UTCL1 misses (profiles/r06/tlb).  The touch is
consumed one stage later (an empty asm with an SGPR input), so the compiler
waits for it there and never leaves it in flight."""
p = "fedavg.hip"
s = open(p).read()


def sub(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new)


sub("    ChunkSrc c0{}, c1{};\n", "    ChunkSrc c0{}, c1{};\n    uint32_t pf = 0;\n")
sub("""        chunk_dma(c0, ki, tiles, dst, lane);
        chunk_dma(c1, ki, tiles, dst + kChunkDma * 256, lane);
""", """        chunk_dma(c0, ki, tiles, dst, lane);
        chunk_dma(c1, ki, tiles, dst + kChunkDma * 256, lane);
        asm volatile("" ::"s"(pf));  // the previous stage's touch has landed
        constexpr int kPf = P2P_XLAT_PF;
        if (ki + kPf < K && c0.bytes) pf = ldc(reinterpret_cast<const uint32_t*>(table_at(c0.peers, ki + kPf) + c0.c0));
""")
sub("constexpr int kAllTilesMaxK = 128;", "#ifndef P2P_XLAT_PF\n#define P2P_XLAT_PF 2\n#endif\nconstexpr int kAllTilesMaxK = 128;")
open(p, "w").write(s)
