#!/usr/bin/env python3
"""Generate register-resident sorting / selection networks for robust.hip.

Each network sorts (or partially sorts) KP uint32 keys held in a fully
unrolled register array.  The base network sorts blocks of 16 with a
60-comparator network and merges them with Batcher's odd-even merges (1447
comparators for 128 against 1471 for Batcher's odd-even merge sort).  For a fixed set of wanted output ranks the network is pruned
backwards: a comparator whose two outputs are both dead is dropped, one with a
single live output becomes a lone v_min_u32 / v_max_u32.

Output: networks.inc (committed; regenerate with `python gen_networks.py`).
Each network is emitted as a device function  net_<tag>(uint32_t (&v)[KP]).

Verification: `python gen_networks.py --check` runs the 0-1 principle
exhaustively for KP <= 16 and on random inputs for every emitted network.
"""
from __future__ import annotations

import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def batcher(n: int):
    """Comparators (lo, hi) of Batcher's odd-even merge sort, n a power of 2."""
    comps = []
    p = 1
    while p < n:
        k = p
        while k >= 1:
            for j in range(k % p, n - k, 2 * k):
                for i in range(min(k, n - j - k)):
                    if (i + j) // (2 * p) == (i + j + k) // (2 * p):
                        comps.append((i + j, i + j + k))
            k //= 2
        p *= 2
    return comps


# A 16-input sorting network of 60 comparators in 10 layers (Green's count;
# Batcher's odd-even merge sort needs 63), checked exhaustively on all 2^16
# 0-1 inputs by --check.
GREEN16 = [
    [(0, 13), (1, 12), (2, 15), (3, 14), (4, 8), (5, 6), (7, 11), (9, 10)],
    [(0, 5), (1, 7), (2, 9), (3, 4), (6, 13), (8, 14), (10, 15), (11, 12)],
    [(0, 1), (2, 3), (4, 5), (6, 8), (7, 9), (10, 11), (12, 13), (14, 15)],
    [(0, 2), (1, 3), (4, 10), (5, 11), (6, 7), (8, 9), (12, 14), (13, 15)],
    [(1, 2), (3, 12), (4, 6), (5, 7), (8, 10), (9, 11), (13, 14)],
    [(1, 4), (2, 6), (5, 8), (7, 10), (9, 13), (11, 14)],
    [(2, 4), (3, 6), (9, 12), (11, 13)],
    [(3, 5), (6, 8), (7, 9), (10, 12)],
    [(3, 4), (5, 6), (7, 8), (9, 10), (11, 12)],
    [(6, 7), (8, 9)],
]


def oddeven_merge(lo: int, hi: int, r: int):
    """Batcher's odd-even merge of the two sorted halves of [lo, hi] (hi
    inclusive) taken with stride r."""
    step = 2 * r
    if step < hi - lo:
        yield from oddeven_merge(lo, hi, step)
        yield from oddeven_merge(lo + r, hi, step)
        for i in range(lo + r, hi - r, step):
            yield (i, i + r)
    else:
        yield (lo, lo + r)


def green_batcher(n: int, lo: int = 0):
    """Sort n = 2^k keys at [lo, lo + n): the 60-comparator network on each
    block of 16, then Batcher's odd-even merges (32: 185, 64: 531, 128: 1447
    comparators against 191 / 543 / 1471)."""
    if n <= 8:
        return [(lo + a, lo + b) for a, b in batcher(n)]
    if n == 16:
        return [(lo + a, lo + b) for layer in GREEN16 for a, b in layer]
    h = n // 2
    return green_batcher(h, lo) + green_batcher(h, lo + h) + list(oddeven_merge(lo, lo + n - 1, 1))


def prune(comps, wanted):
    """Backward liveness.  Returns a list of (op, a, b): op in {CE, MIN, MAX}.
    MIN: v[a] = min(v[a], v[b]);  MAX: v[b] = max(v[a], v[b])."""
    live = set(wanted)
    out = []
    for a, b in reversed(comps):
        la, lb = a in live, b in live
        if la and lb:
            out.append(("CE", a, b))
        elif la:
            out.append(("MIN", a, b))
        elif lb:
            out.append(("MAX", a, b))
        else:
            continue
        live.add(a)
        live.add(b)
    out.reverse()
    return out


def apply(ops, vals):
    v = list(vals)
    for op, a, b in ops:
        lo, hi = min(v[a], v[b]), max(v[a], v[b])
        if op == "CE":
            v[a], v[b] = lo, hi
        elif op == "MIN":
            v[a] = lo
        else:
            v[b] = hi
    return v


# (tag, KP, wanted ranks or None for a full sort)
def bitonic_merge(n: int):
    """Comparators sorting a BITONIC sequence of n (power of 2) ascending:
    half-cleaners at distance n/2, n/4, ..., 1."""
    comps = []
    d = n // 2
    while d >= 1:
        for start in range(0, n, 2 * d):
            for i in range(start, start + d):
                comps.append((i, i + d))
        d //= 2
    return comps


NETWORKS = {"batcher": batcher, "bmerge": bitonic_merge, "green": green_batcher}


def network_specs():
    """(tag, KP, wanted ranks or None = full sort, base network).

    One lane sorts at most 128 keys (256 live keys exceed the register file
    and stall the register allocator).  K <= 64 runs one lane per coordinate
    on sort{KP}; K in 65..256 runs a WAVE GROUP (robust.hip): 2 or 4 waves
    each sort 64 keys of the same coordinates (sort64, either direction) and
    merge across waves with LDS half-cleaners + bmerge64.  sort128 and the
    pruned 128-key networks serve the single-lane K in 65..128 variant."""
    specs = []
    for kp in (2, 4, 8, 16, 32, 64, 128):
        specs.append((f"sort{kp}", kp, None, "green"))
    for kp in (32, 64, 128):
        specs.append((f"bmerge{kp}", kp, None, "bmerge"))
    # specialised K == KP instances for the benchmark configurations
    for kp in (64, 128):
        specs.append((f"median{kp}", kp, [(kp - 1) // 2], "green"))
        b = int(0.2 * kp + 1e-9)
        specs.append((f"trim{kp}_b{b}", kp, list(range(b, kp - b)), "green"))
    # trimmed mean of 256 in one lane per coordinate (robust_pair.hip): the
    # lower / upper 128 of the flip of two sorted halves are bitonic; only
    # ranks 51..127 of the lower and 0..76 of the upper (global 128..204) are
    # summed, so each merger is pruned to those ranks.
    specs.append(("bmerge128_r51_127", 128, list(range(51, 128)), "bmerge"))
    specs.append(("bmerge128_r0_76", 128, list(range(0, 77)), "bmerge"))
    return specs


def emit():
    lines = ["// GENERATED by gen_networks.py -- do not edit.",
             "// Sorting networks (60-comparator 16-sorters + Batcher odd-even merges) over keys of type T (uint32 total-order",
             "// keys, or floats where min/max give the same order),",
             "// pruned to the wanted output ranks.  Counts are per coordinate.",
             "// P2P_CE / P2P_MIN / P2P_MAX are defined by the includer in terms of ASC.",
             "#pragma once", ""]
    for tag, kp, wanted, base in network_specs():
        comps = NETWORKS[base](kp)
        ops = prune(comps, wanted if wanted is not None else range(kp))
        nce = sum(1 for o in ops if o[0] == "CE")
        n1 = len(ops) - nce
        lines.append(f"// {tag}: KP={kp} wanted={'all' if wanted is None else f'{wanted[0]}..{wanted[-1]}'}"
                     f" comparators={nce} half-ops={n1} valu={2 * nce + n1}")
        lines.append(f"template <bool ASC, typename T, typename H = NoHook>  // ASC=false sorts descending")
        lines.append(f"__device__ __forceinline__ void net_{tag}(T (&v)[{kp}], H&& hook = H{{}}) {{")
        # hook(v, blk) runs before the first comparator that reads block blk
        # (16 keys) -- the block still holds its inputs there.  A NaN test per
        # block then waits only for that block's loads (robust_nets.h).
        seen = set()
        for op, a, b in ops:
            for blk in sorted({a // 16, b // 16} - seen) if kp >= 16 and base != "bmerge" else ():
                lines.append(f"  hook(v, {blk});")
                seen.add(blk)
            lines.append(f"  P2P_{op}(v[{a}], v[{b}]);")
        lines.append("}")
        lines.append("")
    with open(os.path.join(HERE, "networks.inc"), "w") as f:
        f.write("\n".join(lines))


def check():
    rng = random.Random(1)
    for tag, kp, wanted, base in network_specs():
        ops = prune(NETWORKS[base](kp), wanted if wanted is not None else range(kp))
        want = list(range(kp)) if wanted is None else wanted
        if base == "bmerge":  # input domain: bitonic sequences (asc ++ desc, rotated)
            def bitonic(vals):
                h = rng.randrange(kp + 1)
                s = sorted(vals[:h]) + sorted(vals[h:], reverse=True)
                r = rng.randrange(kp)
                return s[r:] + s[:r]
            inputs = [bitonic([rng.randrange(m) for _ in range(kp)]) for m in (2, 3, 1 << 32) for _ in range(2000)]
            want = list(range(kp)) if wanted is None else wanted
            for vals in inputs:
                got, ref = apply(ops, vals), sorted(vals)
                assert all(got[r] == ref[r] for r in want), (tag, vals)
            print(f"{tag}: ok ({len(ops)} ops)")
            continue
        if kp <= 16:
            inputs = ([(m >> i) & 1 for i in range(kp)] for m in range(1 << kp))
        else:
            inputs = ([rng.randrange(4) for _ in range(kp)] for _ in range(3000))
        for vals in inputs:
            got = apply(ops, vals)
            ref = sorted(vals)
            assert all(got[r] == ref[r] for r in want), (tag, vals)
        for _ in range(300):
            vals = [rng.randrange(1 << 32) for _ in range(kp)]
            got, ref = apply(ops, vals), sorted(vals)
            assert all(got[r] == ref[r] for r in want), tag
        print(f"{tag}: ok ({len(ops)} ops)")


if __name__ == "__main__":
    if "--check" in sys.argv:
        check()
    else:
        emit()
