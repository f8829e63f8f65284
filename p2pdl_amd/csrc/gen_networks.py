#!/usr/bin/env python3
"""Generate register-resident sorting / selection networks for the robust kernels.

Each network sorts (or partially sorts) KP keys held in a fully unrolled
register array: Batcher's odd-even merge sort, or a bitonic merger for the
flip of two sorted lists.  For a fixed set of wanted output ranks the network
is pruned backwards: a comparator whose two outputs are both dead is dropped,
one with a single live output becomes a lone min or max.

Three-input lowering (round 3).  A comparator network issues one VALU
instruction per comparator output.  gfx950 has full-rate three-input
v_min3 / v_max3 / v_med3 (f32 and u32), so a min or max whose every consumer
can take its two operands directly need not be computed at all:
  min(o, min(x, y)) = min3(o, x, y)                  always
  max(o, max(x, y)) = max3(o, x, y)                  always
  max(o, min(x, y)) = med3(o, x, y)   iff o <= max(x, y) on every input
  min(o, max(x, y)) = med3(o, x, y)   iff o >= min(x, y) on every input
The two conditional forms are decided by the 0-1 principle on the input
domain of the network stage both nodes belong to (all 0-1 vectors for a
16-sorter, two sorted 0-1 halves for an odd-even merge, 0-1 bitonic
sequences for a bitonic merger): min, max and med3 commute with every
threshold map, so a relation that holds on all thresholded inputs holds on
all inputs.  Pruned networks are checked on the same domains -- every live
value is computed exactly as in the unpruned network.  A greedy pass from the
outputs backwards eliminates a node when all its consumers can absorb it (each
consumer absorbs at most one operand, and an eliminated node's operands must
themselves be computed); an exact MILP of the same selection problem finds
at most 0.7% more.  sort128: 2942 -> 2184 VALU (round 2's 16-block network:
2894), bmerge128 pruned to ranks 51..127: 619 -> 430.

Output: networks.inc (committed; regenerate with `python gen_networks.py`;
`--classic` writes the round-2 two-input form, for A/B builds only).
Each network is emitted as a device function  net_<tag><ASC>(T (&v)[KP], hook).

Verification: `python gen_networks.py --check` runs every emitted program
(the instruction list as emitted, three-input ops included) on 0-1 inputs --
exhaustively for KP <= 16, on every domain vector of a bitonic merger -- and
on random 32-bit inputs, against sorted().
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


# A stage of a network: (kind, first wire, width).  Its input domain decides
# the conditional med3 forms (domain()).
def green_batcher(n: int, lo: int = 0):
    """Sort n = 2^k keys at [lo, lo + n): the 60-comparator network on each
    block of 16, then Batcher's odd-even merges (32: 185, 64: 531, 128: 1447
    comparators against 191 / 543 / 1471).  Returns ((a, b), stage) pairs."""
    if n <= 8:
        return [((lo + a, lo + b), ("all", lo, n)) for a, b in batcher(n)]
    if n == 16:
        return [((lo + a, lo + b), ("all", lo, 16)) for layer in GREEN16 for a, b in layer]
    h = n // 2
    return (green_batcher(h, lo) + green_batcher(h, lo + h)
            + [(c, ("merge", lo, n)) for c in oddeven_merge(lo, lo + n - 1, 1)])


def batcher_stages(n: int, lo: int = 0):
    """Batcher's odd-even merge sort of [lo, lo + n), each merge its own
    stage (two sorted halves in).  More comparators than green_batcher's
    16-blocks (1471 against 1447 for 128) but fewer instructions once
    lowered to three-input forms (2184 against 2248): the 16-sorter's
    irregular layers leave fewer minima / maxima for a consumer to absorb."""
    if n == 1:
        return []
    if n == 4:  # the three-input 4-sorter (7 instructions; Batcher's 5 comparators lower to 9)
        return [((lo, lo + 1, lo + 2, lo + 3), ("all", lo, 4))]
    h = n // 2
    return (batcher_stages(h, lo) + batcher_stages(h, lo + h)
            + [(c, ("merge", lo, n)) for c in oddeven_merge(lo, lo + n - 1, 1)])


def bitonic_merge(n: int):
    """Comparators sorting a BITONIC sequence of n (power of 2) ascending:
    half-cleaners at distance n/2, n/4, ..., 1."""
    comps = []
    d = n // 2
    while d >= 1:
        for start in range(0, n, 2 * d):
            for i in range(start, start + d):
                comps.append(((i, i + d), ("bitonic", 0, n)))
        d //= 2
    return comps


# base network per emission form: "sort" is Batcher's merge sort when lowered
# to three-input forms, the 16-block network in the round-2 (--classic) form
def merge_stage(n: int):
    """Batcher's odd-even merge of the two sorted halves of n keys."""
    return [(c, ("merge", 0, n)) for c in oddeven_merge(0, n - 1, 1)]


NETWORKS = {"bmerge": bitonic_merge, "sort": batcher_stages, "merge": merge_stage}
CLASSIC = {"bmerge": bitonic_merge, "sort": green_batcher, "merge": merge_stage}


def domain(stage):
    """The 0-1 input vectors of a stage (over its own wires)."""
    kind, _, n = stage
    if kind == "all":
        return [[(m >> i) & 1 for i in range(n)] for m in range(1 << n)]
    if kind == "merge":  # two sorted halves
        h = n // 2
        return [[0] * (h - i) + [1] * i + [0] * (h - j) + [1] * j for i in range(h + 1) for j in range(h + 1)]
    if kind == "bitonic":  # 0^a 1^b 0^c and 1^a 0^b 1^c (every cyclic rotation of up-then-down)
        out = set()
        for a in range(n + 1):
            for b in range(n + 1 - a):
                c = n - a - b
                out.add((0,) * a + (1,) * b + (0,) * c)
                out.add((1,) * a + (0,) * b + (1,) * c)
        return [list(x) for x in sorted(out)]
    raise ValueError(kind)


_DOMAIN_BITS = {}


def domain_bits(kind, n):
    """Per wire of a stage, its values over the stage's domain as one integer
    (bit s = the wire's value on domain vector s)."""
    import numpy as np

    if (kind, n) not in _DOMAIN_BITS:
        dom = np.array(domain((kind, 0, n)), dtype=np.uint8)
        _DOMAIN_BITS[(kind, n)] = [int.from_bytes(np.packbits(dom[:, j], bitorder="little").tobytes(), "little")
                                   for j in range(n)]
    return _DOMAIN_BITS[(kind, n)]


def prune(tagged, wanted):
    """Backward liveness.  Returns ((op, a, b), stage) with op in {CE, MIN, MAX}.
    MIN: v[a] = min(v[a], v[b]);  MAX: v[b] = max(v[a], v[b]).  A 4-sorter
    ((a, b, c, d), stage) stays whole while any of its outputs is live (its
    dead outputs are dropped later, by the SSA liveness of Program)."""
    live = set(wanted)
    out = []
    for wires, st in reversed(tagged):
        if len(wires) == 4:
            if live.intersection(wires):
                out.append((("SORT4",) + tuple(wires), st))
                live.update(wires)
            continue
        a, b = wires
        la, lb = a in live, b in live
        if la and lb:
            out.append((("CE", a, b), st))
        elif la:
            out.append((("MIN", a, b), st))
        elif lb:
            out.append((("MAX", a, b), st))
        else:
            continue
        live.add(a)
        live.add(b)
    out.reverse()
    return out


def apply(ops, vals):
    """Runs a pruned comparator list (classic form) on vals."""
    v = list(vals)
    for op_, _ in ops:
        if op_[0] == "SORT4":
            w = op_[1:]
            for i, x in zip(w, sorted(v[j] for j in w)):
                v[i] = x
            continue
        op, a, b = op_
        lo, hi = min(v[a], v[b]), max(v[a], v[b])
        if op == "CE":
            v[a], v[b] = lo, hi
        elif op == "MIN":
            v[a] = lo
        else:
            v[b] = hi
    return v


class Program:
    """A network as SSA nodes: 0..kp-1 the inputs v[i]; then ("lo"|"hi", x, y)
    for min / max, lowered to three-input forms by fuse()."""

    def __init__(self, ops, kp, wanted):
        self.kp = kp
        self.kind = ["in"] * kp
        self.args = [()] * kp
        self.stage = [None] * kp
        wire = list(range(kp))
        for op_, st in ops:
            if op_[0] == "SORT4":  # sort3(a, b, c), then d inserted by med3
                a, b, c, d = (wire[w] for w in op_[1:])
                t0 = self._node("lo3", (a, b, c), st)
                t1 = self._node("med3", (a, b, c), st)
                t2 = self._node("hi3", (a, b, c), st)
                ys = (self._node("lo", (t0, d), st), self._node("med3", (t0, t1, d), st),
                      self._node("med3", (t1, t2, d), st), self._node("hi", (t2, d), st))
                for w, y in zip(op_[1:], ys):
                    wire[w] = y
                continue
            op, a, b = op_
            va, vb = wire[a], wire[b]
            if op in ("CE", "MIN"):
                wire[a] = self._node("lo", (va, vb), st)
            if op in ("CE", "MAX"):
                wire[b] = self._node("hi", (va, vb), st)
        self.out = {w: wire[w] for w in wanted}
        live = set(self.out.values())
        for i in range(len(self.kind) - 1, -1, -1):
            if i in live:
                live.update(self.args[i])
        self.live = live
        # the values every stage sees, as bitsets over its domain: bit s of
        # bits[node] = the node's value on domain vector s
        self.bits = {}
        stage_in = {}
        wire = list(range(kp))
        node = kp
        for op_, st in ops:
            stage_in.setdefault(st, list(wire))
            if op_[0] == "SORT4":
                for k, w in enumerate(op_[1:]):
                    wire[w] = node + 3 + k
                node += 7
                continue
            op, a, b = op_
            if op in ("CE", "MIN"):
                wire[a] = node
                node += 1
            if op in ("CE", "MAX"):
                wire[b] = node
                node += 1
        for st, w in stage_in.items():
            _, lo, n = st
            b = {w[lo + j]: m for j, m in enumerate(domain_bits(st[0], n))}
            for i in range(kp, len(self.kind)):
                if self.stage[i] == st:
                    xs = [b[a] for a in self.args[i]]
                    k = self.kind[i]
                    if k in ("lo", "lo3"):
                        b[i] = xs[0] & xs[1] & (xs[2] if len(xs) > 2 else -1)
                    elif k in ("hi", "hi3"):
                        b[i] = xs[0] | xs[1] | (xs[2] if len(xs) > 2 else 0)
                    else:  # med3 = majority
                        b[i] = (xs[0] & xs[1]) | (xs[0] & xs[2]) | (xs[1] & xs[2])
            self.bits[st] = b
        self.absorbed = {}  # consumer -> the operand node it absorbs
        self.elim = set()

    def _node(self, kind, args, st):
        self.kind.append(kind)
        self.args.append(args)
        self.stage.append(st)
        return len(self.kind) - 1

    def can_absorb(self, c, e):
        f, g = self.kind[c], self.kind[e]
        if f == g:
            return True  # min of a min / max of a max
        st = self.stage[c]
        if st is None or st != self.stage[e]:
            return False
        (o,) = [a for a in self.args[c] if a != e] or [None]
        if o is None:
            return False
        b = self.bits[st]
        x, y = self.args[e]
        if f == "hi":  # max(o, min(x, y)) = med3 iff o <= max(x, y)
            return b[o] & ~(b[x] | b[y]) == 0
        return (b[x] & b[y]) & ~b[o] == 0  # min(o, max(x, y)) = med3 iff o >= min(x, y)

    def fuse(self, reverse=True):
        cons = {i: [] for i in range(len(self.kind))}
        for i in self.live:
            for a in self.args[i]:
                cons[a].append(i)
        outs = set(self.out.values())
        must = set()
        order = sorted(i for i in self.live if self.kind[i] != "in")
        for e in (reversed(order) if reverse else order):
            if e in outs or e in must or e in self.absorbed or not cons[e]:
                continue
            if self.kind[e] not in ("lo", "hi") or any(self.kind[c] not in ("lo", "hi") for c in cons[e]):
                continue  # a three-input node can neither be absorbed nor absorb
            if any(c in self.absorbed or c in self.elim for c in cons[e]):
                continue
            if any(a in self.elim for a in self.args[e]):
                continue
            if not all(self.can_absorb(c, e) for c in cons[e]):
                continue
            self.elim.add(e)
            for c in cons[e]:
                self.absorbed[c] = e
            must.update(self.args[e])
        return self

    def instrs(self):
        if getattr(self, "_ins", None) is None:
            self._ins = self._lower()
        return self._ins

    def _lower(self):
        """[(node, op, operands)]: op in lo, hi, lo3, hi3, med3; for a `hi` whose
        sibling `lo` of the same operands is computed, the sibling rides along
        (kx / fx take max as a ^ b ^ min)."""
        out = []
        lo_of = {}
        for i in sorted(self.live):
            if self.kind[i] == "in" or i in self.elim:
                continue
            if self.kind[i] in ("lo3", "hi3", "med3"):
                out.append((i, self.kind[i], self.args[i]))
                continue
            if i in self.absorbed:
                e = self.absorbed[i]
                (o,) = [a for a in self.args[i] if a != e]
                x, y = self.args[e]
                op = self.kind[i] + "3" if self.kind[i] == self.kind[e] else "med3"
                out.append((i, op, (o, x, y)))
            else:
                x, y = self.args[i]
                if self.kind[i] == "lo":
                    lo_of[(x, y)] = i
                    out.append((i, "lo", (x, y)))
                else:
                    out.append((i, "hi", (x, y, lo_of.get((x, y)))))
        return out

    def run(self, vals):
        """The emitted program on a batch of inputs (rows of vals, ascending
        order); returns the final wires."""
        import numpy as np

        vals = np.asarray(vals)
        val = {i: vals[:, i] for i in range(self.kp)}
        for i, op, a in self.instrs():
            x, y = val[a[0]], val[a[1]]
            if op == "lo":
                val[i] = np.minimum(x, y)
            elif op == "hi":
                val[i] = np.maximum(x, y)
            else:
                z = val[a[2]]
                lo, hi = np.minimum(x, y), np.maximum(x, y)
                val[i] = (np.minimum(lo, z) if op == "lo3" else np.maximum(hi, z) if op == "hi3"
                          else np.maximum(lo, np.minimum(hi, z)))
        res = vals.copy()
        for w, n in self.out.items():
            res[:, w] = val[n]
        return res


def network_specs():
    """(tag, KP, wanted ranks or None = full sort, base network).

    One lane sorts at most 128 keys (256 live keys exceed the register file).
    sort{KP} serve the one-lane kernels (robust.hip), the four-list median,
    the pair kernels (robust_pair.hip) and the 4-lane LDS kernels
    (robust_lds.hip, either direction, bmerge64 across lanes)."""
    specs = []
    for kp in (2, 4, 8, 16, 32, 64, 128):
        specs.append((f"sort{kp}", kp, None, "sort"))
    for kp in (32, 64, 128):
        specs.append((f"bmerge{kp}", kp, None, "bmerge"))
    # specialised K == KP instances for the benchmark configurations
    for kp in (64, 128):
        specs.append((f"median{kp}", kp, [(kp - 1) // 2], "sort"))
        b = int(0.2 * kp + 1e-9)
        specs.append((f"trim{kp}_b{b}", kp, list(range(b, kp - b)), "sort"))
    # trimmed mean of 256 (robust_pair.hip): Batcher's odd-even merge of the
    # two waves' sorted 128 split by parity -- v = merge(A_even, B_even) in
    # wave 0, w = merge(A_odd, B_odd) in wave 1; ranks 51..204 of the merge
    # need v_26..v_102 and w_25..w_101.  (bmerge128: the flip variant's
    # mergers, for the 4-lane LDS kernels' cross-lane form.)
    specs.append(("merge128_r26_102", 128, list(range(26, 103)), "merge"))
    specs.append(("merge128_r25_101", 128, list(range(25, 102)), "merge"))
    return specs


def build(tag, kp, wanted, base):
    ops = prune(NETWORKS[base](kp), wanted if wanted is not None else range(kp))
    want = list(range(kp)) if wanted is None else wanted
    # the better of a backward and a forward greedy pass
    best = min((Program(ops, kp, want).fuse(reverse=r) for r in (True, False)), key=lambda p: len(p.instrs()))
    return ops, best


HEADER = ["// GENERATED by gen_networks.py -- do not edit.",
          "// Sorting networks (Batcher odd-even merge sorts, or bitonic mergers) over",
          "// values of type T (uint32 total-order keys, or floats where min / max give the same order),",
          "// pruned to the wanted output ranks.  Counts are per coordinate."]


def emit_classic():
    lines = HEADER + ["// P2P_CE / P2P_MIN / P2P_MAX are defined by the includer in terms of ASC.", "#pragma once", ""]
    for tag, kp, wanted, base in network_specs():
        ops = prune(CLASSIC[base](kp), wanted if wanted is not None else range(kp))
        nce = sum(1 for (o, _, _), _ in ops if o == "CE")
        n1 = len(ops) - nce
        lines.append(f"// {tag}: KP={kp} wanted={'all' if wanted is None else f'{wanted[0]}..{wanted[-1]}'}"
                     f" comparators={nce} half-ops={n1} valu={2 * nce + n1}")
        lines.append("template <bool ASC, typename T, typename H = NoHook>  // ASC=false sorts descending")
        lines.append(f"__device__ __forceinline__ void net_{tag}(T (&v)[{kp}], H&& hook = H{{}}) {{")
        seen = set()
        for (op, a, b), _ in ops:
            for blk in sorted({a // 16, b // 16} - seen) if kp >= 16 and base == "sort" else ():
                lines.append(f"  hook(v, {blk});")
                seen.add(blk)
            lines.append(f"  P2P_{op}(v[{a}], v[{b}]);")
        lines.append("}")
        lines.append("")
    return lines


def emit_fused():
    lines = HEADER + [
        "// Lowered to one instruction per computed value: P2P_LO / P2P_HI (two inputs; P2P_HIS also gets the",
        "// sibling min of the same operands), P2P_LO3 / P2P_HI3 / P2P_MED3 (three inputs) -- defined by the",
        "// includer in terms of ASC (robust_nets.h).  Inputs are read from v, results written back at the end.",
        "#pragma once", ""]
    for tag, kp, wanted, base in network_specs():
        ops, prog = build(tag, kp, wanted, base)
        ins = prog.instrs()
        nce = sum(1 for o, _ in ops if o[0] == "CE") + 5 * sum(1 for o, _ in ops if o[0] == "SORT4")
        cnt = {k: sum(1 for _, op, _ in ins if op == k) for k in ("lo3", "hi3", "med3")}
        lines.append(f"// {tag}: KP={kp} wanted={'all' if wanted is None else f'{wanted[0]}..{wanted[-1]}'}"
                     f" comparators={nce} two-input valu={2 * nce + sum(1 for o, _ in ops if o[0] in ('MIN', 'MAX'))} -> {len(ins)}"
                     f" (min3 {cnt['lo3']}, max3 {cnt['hi3']}, med3 {cnt['med3']})")
        lines.append("template <bool ASC, typename T, typename H = NoHook>  // ASC=false sorts descending")
        lines.append(f"__device__ __forceinline__ void net_{tag}(T (&v)[{kp}], H&& hook = H{{}}) {{")

        def ref(n):
            return f"v[{n}]" if n < kp else f"n{n}"

        seen = set()
        for i, op, a in ins:
            # hook(v, blk) runs before the first instruction that reads input
            # block blk (16 keys) -- v still holds the inputs there
            blks = {x // 16 for x in a if x is not None and x < kp}
            for blk in sorted(blks - seen) if kp >= 16 and base == "sort" else ():
                lines.append(f"  hook(v, {blk});")
                seen.add(blk)
            if op == "lo":
                rhs = f"P2P_LO({ref(a[0])}, {ref(a[1])})"
            elif op == "hi":
                rhs = (f"P2P_HIS({ref(a[0])}, {ref(a[1])}, {ref(a[2])})" if a[2] is not None
                       else f"P2P_HI({ref(a[0])}, {ref(a[1])})")
            else:
                rhs = f"P2P_{op.upper()}({ref(a[0])}, {ref(a[1])}, {ref(a[2])})"
            lines.append(f"  const T n{i} = {rhs};")
        for w in sorted(prog.out):
            if prog.out[w] >= kp:
                lines.append(f"  v[{w}] = n{prog.out[w]};")
        lines.append("}")
        lines.append("")
    return lines


def check():
    import numpy as np

    rng = np.random.default_rng(1)
    for tag, kp, wanted, base in network_specs():
        ops, prog = build(tag, kp, wanted, base)
        want = list(range(kp)) if wanted is None else wanted
        if base == "bmerge":  # every 0-1 bitonic vector, and bitonic sequences of random values
            rows = [np.array(domain(("bitonic", 0, kp)), dtype=np.uint64)]
            for m in (3, 1 << 32):
                x = rng.integers(0, m, size=(2000, kp), dtype=np.uint64)
                h = rng.integers(0, kp + 1, size=2000)
                for r in range(2000):  # ascending then descending, rotated
                    s = np.concatenate([np.sort(x[r, :h[r]]), np.sort(x[r, h[r]:])[::-1]])
                    x[r] = np.roll(s, int(rng.integers(kp)))
                rows.append(x)
            inputs = np.concatenate(rows)
        elif base == "merge":  # every 0-1 pair of sorted halves, and sorted halves of random values
            rows = [np.array(domain(("merge", 0, kp)), dtype=np.uint64)]
            for m in (3, 1 << 32):
                x = rng.integers(0, m, size=(3000, kp), dtype=np.uint64)
                rows.append(np.concatenate([np.sort(x[:, :kp // 2], axis=1), np.sort(x[:, kp // 2:], axis=1)], axis=1))
            inputs = np.concatenate(rows)
        elif kp <= 16:
            m = np.arange(1 << kp, dtype=np.uint64)
            inputs = (m[:, None] >> np.arange(kp, dtype=np.uint64)[None, :]) & np.uint64(1)
        else:
            inputs = np.concatenate([rng.integers(0, m, size=(4000, kp), dtype=np.uint64) for m in (2, 4, 1 << 32)])
        ref = np.sort(inputs, axis=1)[:, want]
        fused = prog.run(inputs)[:, want]
        assert np.array_equal(fused, ref), (tag, "fused")
        for vals in inputs[:: max(1, len(inputs) // 300)].tolist():  # the classic form, spot-checked
            got, srt = apply(ops, vals), sorted(vals)
            assert all(got[r] == srt[r] for r in want), (tag, "classic", vals)
        print(f"{tag}: ok ({len(ops)} comparators, {len(prog.instrs())} instructions, {len(inputs)} inputs)")


if __name__ == "__main__":
    if "--check" in sys.argv:
        check()
    else:
        lines = emit_classic() if "--classic" in sys.argv else emit_fused()
        with open(os.path.join(HERE, "networks.inc"), "w") as f:
            f.write("\n".join(lines))
