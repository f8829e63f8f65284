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

Three-list merges (round 4, MSort below): the sorts are trees of merges of
THREE sorted lists whose cleanup is one three-input operation per output --
sort128 1962 instead of 2120 (Batcher lowered), sort64 731 / 789, median128
1370 / 1658, trim128 1786 / 1976; the pruned parity mergers of the K = 256
trimmed mean split by index modulo 3 (390 / 398).

Output: networks.inc (committed; regenerate with `python gen_networks.py`;
`--classic` writes the round-2 two-input form, for A/B builds only).
Each network is emitted as a device function  net_<tag><ASC>(T (&v)[KP], hook).

Verification: every MSort stage asserts each output against its rank on the
stage's whole 0-1 domain as it is built (a proof by the 0-1 principle: min,
max and med3 commute with thresholds).  `python gen_networks.py --check`
runs every emitted program
(the instruction list as emitted, three-input ops included) on 0-1 inputs --
exhaustively for KP <= 16, on every domain vector of a bitonic merger -- and
on random 32-bit inputs, against sorted().
"""
from __future__ import annotations

import itertools
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


# ---- Three-list merge sort ("msort", round 4) --------------------------------
# Batcher's merge splits two sorted lists by index parity, merges the classes
# and fixes the interleaving with one layer of comparators.  The same scheme
# works for THREE sorted lists: split each by parity, merge the three even
# classes and the three odd classes (recursively), interleave, and every
# output of the merge is then ONE min / max / min3 / max3 / med3 of the
# interleaved values in a window of +-6 around its rank (found by search and
# proved on the stage's 0-1 domain: all combinations of the lists' zero
# counts).  Four lists do not close with one operation per output.  A sort
# tree of three-list merges (MSORT_TREE, from `--search`: the lowered
# instruction count of every candidate split) sorts 128 keys in 1962
# instructions against 2120 for the lowered Batcher sort, 64 in 731 / 789.
# Every stage is built as SSA nodes with their values on that stage's domain,
# so Program's three-input absorption applies unchanged.
MSORT_TREE = {128: (43, 43, 42), 64: (22, 21, 21), 43: (15, 14, 14), 42: (14, 14, 14), 32: (12, 10, 10),
              22: (8, 7, 7), 21: (9, 6, 6), 16: (9, 7), 15: (9, 6), 14: (9, 5), 12: (4, 4, 4), 10: (4, 3, 3),
              9: (3, 3, 3), 8: (3, 3, 2), 7: (4, 3), 6: (3, 3), 5: (3, 2)}
MSORT_WINDOW = 6


def _pack(mask) -> int:
    """A numpy bool vector as an int bitset (bit s = element s)."""
    import numpy as np

    return int.from_bytes(np.packbits(mask, bitorder="little").tobytes(), "little")


class MSort:
    """SSA nodes of a three-list merge sort: kind / args / stage per node as in
    Program; bits[stage][node] = the node's values on the stage's 0-1 domain."""

    def __init__(self, kp: int):
        self.kp = kp
        self.kind = ["in"] * kp
        self.args = [()] * kp
        self.stage = [None] * kp
        self.bits = {}

    def _op(self, st, kind, args, cache):
        key = (kind, tuple(sorted(args)))
        if key in cache:
            return cache[key]
        b = self.bits[st]
        xs = [b[a] for a in key[1]]
        if kind in ("lo", "lo3"):
            m = xs[0] & xs[1] & (xs[2] if len(xs) > 2 else -1)
        elif kind in ("hi", "hi3"):
            m = xs[0] | xs[1] | (xs[2] if len(xs) > 2 else 0)
        else:  # med3 = majority
            m = (xs[0] & xs[1]) | (xs[0] & xs[2]) | (xs[1] & xs[2])
        self.kind.append(kind)
        self.args.append(key[1])
        self.stage.append(st)
        i = len(self.kind) - 1
        b[i] = m
        cache[key] = i
        return i

    def sort(self, wires, tree=None):
        tree = MSORT_TREE if tree is None else tree
        n = len(wires)
        if n <= 4:
            return self.merge([[w] for w in wires])
        lists, i = [], 0
        for part in tree[n]:
            lists.append(self.sort(wires[i:i + part], tree))
            i += part
        return self.merge(lists)

    def merge(self, lists, k=2, win=MSORT_WINDOW):
        """One stage: merge 2-4 sorted node lists (4 only of single nodes),
        splitting by index modulo k (an int, or a function of the longest
        list's length).  Returns the output nodes, each checked against its
        rank on the whole 0-1 domain of the stage."""
        import numpy as np

        st = ("mmerge", len(self.bits))
        sizes = [len(x) for x in lists]
        zs = [g.reshape(-1) for g in np.meshgrid(*[np.arange(s + 1) for s in sizes], indexing="ij")]
        b = self.bits[st] = {}
        for z, lst in zip(zs, lists):
            for j, x in enumerate(lst):
                b[x] = _pack(z <= j)  # a sorted 0-1 list with z zeros: element j is 1 iff j >= z
        out = self._merge(st, list(lists), zs, k, win, {})
        total = sum(zs)
        assert all(b[x] == _pack(total <= t) for t, x in enumerate(out)), (st, sizes)
        return out

    def _merge(self, st, lists, zs, k, win, cache):
        import numpy as np

        pairs = [(lst, z) for lst, z in zip(lists, zs) if lst]
        lists, zs = [p[0] for p in pairs], [p[1] for p in pairs]
        op = lambda kind, *a: self._op(st, kind, a, cache)  # noqa: E731
        if len(lists) == 1:
            return list(lists[0])
        if all(len(x) == 1 for x in lists):
            v = [x[0] for x in lists]
            if len(v) == 2:
                return [op("lo", *v), op("hi", *v)]
            if len(v) == 3:
                return [op("lo3", *v), op("med3", *v), op("hi3", *v)]
            a, b_, c, d = v  # sort3, then d inserted by med3 (7 instructions)
            t0, t1, t2 = op("lo3", a, b_, c), op("med3", a, b_, c), op("hi3", a, b_, c)
            return [op("lo", t0, d), op("med3", t0, t1, d), op("med3", t1, t2, d), op("hi", t2, d)]
        if len(lists) == 2 and min(len(x) for x in lists) == 1:  # insertion: n + 1 (optimal)
            big, one = (lists[0], lists[1][0]) if len(lists[1]) == 1 else (lists[1], lists[0][0])
            return ([op("lo", big[0], one)] + [op("med3", big[i - 1], big[i], one) for i in range(1, len(big))]
                    + [op("hi", big[-1], one)])
        assert len(lists) <= 3, "four lists do not close with one operation per output"
        longest = max(len(x) for x in lists)
        kk = min(k(longest) if callable(k) else k, longest)
        subs = []
        for r in range(kk):  # class r of every list: its zero count is ceil((z - r) / kk)
            subs.append(self._merge(st, [x[r::kk] for x in lists],
                                    [np.maximum(0, (z - r + kk - 1) // kk) for z in zs], k, win, cache))
        seq = [subs[r][i] for i in range(max(map(len, subs))) for r in range(kk) if i < len(subs[r])]
        total = sum(zs)
        b = self.bits[st]
        out = []
        for t in range(len(seq)):
            want = _pack(total <= t)
            pos = range(max(0, t - win), min(len(seq), t + win + 1))
            f = next((seq[i] for i in pos if b[seq[i]] == want), None)
            if f is None:
                for i, j in itertools.combinations(pos, 2):
                    x, y = b[seq[i]], b[seq[j]]
                    if x & y == want or x | y == want:
                        f = op("lo" if x & y == want else "hi", seq[i], seq[j])
                        break
            if f is None:
                for i, j, l in itertools.combinations(pos, 3):
                    x, y, z = b[seq[i]], b[seq[j]], b[seq[l]]
                    kind = ("lo3" if x & y & z == want else "hi3" if x | y | z == want
                            else "med3" if (x & y) | (x & z) | (y & z) == want else None)
                    if kind:
                        f = op(kind, seq[i], seq[j], seq[l])
                        break
            if f is None:
                raise ValueError(f"no one-operation output for rank {t} of a merge of {[len(x) for x in lists]}")
            out.append(f)
        return out


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
CLASSIC = {"bmerge": bitonic_merge, "sort": green_batcher, "msort": green_batcher, "merge": merge_stage}


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


class MSortProgram(Program):
    """Program over an MSort network, pruned to the wanted ranks by liveness."""

    def __init__(self, kp, wanted, tree=None, net=None):
        if net is None:
            net = MSort(kp)
            outs = net.sort(list(range(kp)), tree)
        else:
            net, outs = net
        self.kp = kp
        self.kind, self.args, self.stage, self.bits = net.kind, net.args, net.stage, net.bits
        self.out = {w: outs[w] for w in wanted}
        live = set(self.out.values())
        for i in range(len(self.kind) - 1, -1, -1):
            if i in live:
                live.update(self.args[i])
        self.live = live
        self.absorbed = {}
        self.elim = set()
        self._ins = None


def merge_cost(sizes, k=2) -> int:
    """Lowered instruction count of one merge stage of sorted lists of `sizes`."""
    n = sum(sizes)
    net = MSort(n)
    lists, i = [], 0
    for s in sizes:
        lists.append(list(range(i, i + s)))
        i += s
    outs = net.merge(lists, k)
    return min(len(MSortProgram(n, range(n), net=(net, outs)).fuse(reverse=r).instrs()) for r in (True, False))


def search_tree(sizes=(128, 64, 32, 16, 8), spread=2, wide_below=0, wide=6):
    """The MSORT_TREE search: for each n the cheapest split into two or three
    near-balanced parts (each part up to `spread` above the balanced size;
    `wide` for n <= wide_below), scored by lowered instruction counts."""
    import functools

    @functools.lru_cache(None)
    def mc(parts):
        try:
            return merge_cost(parts)
        except (ValueError, AssertionError):
            return None

    @functools.lru_cache(None)
    def best(n):
        if n <= 4:
            return ({1: 0, 2: 2, 3: 3, 4: 7}[n], None)
        cands = []
        sp = wide if n <= wide_below else spread
        for a in range((n + 1) // 2, min(n - 1, (n + 1) // 2 + sp) + 1):
            cands.append((a, n - a))
        for a in range(-(-n // 3), -(-n // 3) + sp + 1):
            for b2 in range(-(-(n - a) // 2), -(-(n - a) // 2) + sp):
                c = n - a - b2
                if 1 <= c <= b2 <= a:
                    cands.append((a, b2, c))
        top = None
        for parts in cands:
            m = mc(parts)
            if m is None:
                continue
            tot = m + sum(best(x)[0] for x in parts)
            if top is None or tot < top[0]:
                top = (tot, parts)
        return top

    for n in sizes:
        print(n, best(n), flush=True)
    tree = {}

    def walk(n):
        parts = best(n)[1]
        if parts:
            tree[n] = parts
            for x in parts:
                walk(x)

    for n in sizes:
        walk(n)
    print("MSORT_TREE =", dict(sorted(tree.items(), reverse=True)))


def network_specs():
    """(tag, KP, wanted ranks or None = full sort, base network).

    One lane sorts at most 128 keys (256 live keys exceed the register file).
    sort{KP} serve the one-lane kernels (robust.hip), the four-list median,
    the pair kernels (robust_pair.hip) and the 4-lane LDS kernels
    (robust_lds.hip, either direction, bmerge64 across lanes)."""
    specs = []
    for kp in (2, 4, 8, 16, 32, 64, 128):
        specs.append((f"sort{kp}", kp, None, "msort"))
    for kp in (32, 64, 128):
        specs.append((f"bmerge{kp}", kp, None, "bmerge"))
    # specialised K == KP instances for the benchmark configurations
    for kp in (64, 128):
        specs.append((f"median{kp}", kp, [(kp - 1) // 2], "msort"))
        b = int(0.2 * kp + 1e-9)
        specs.append((f"trim{kp}_b{b}", kp, list(range(b, kp - b)), "msort"))
    # trimmed mean of 256 (robust_pair.hip): Batcher's odd-even merge of the
    # two waves' sorted 128 split by parity -- v = merge(A_even, B_even) in
    # wave 0, w = merge(A_odd, B_odd) in wave 1; ranks 51..204 of the merge
    # need v_26..v_102 and w_25..w_101.  (bmerge128: the flip variant's
    # mergers, for the 4-lane LDS kernels' cross-lane form.)
    specs.append(("merge128_r26_102", 128, list(range(26, 103)), "merge"))
    specs.append(("merge128_r25_101", 128, list(range(25, 102)), "merge"))
    return specs


_MSORT_NETS = {}


def build(tag, kp, wanted, base):
    """(comparator list or None, lowered Program).  "msort": the three-list
    merge sort, or Batcher's lowered sort where that is shorter (pruned specs
    can go either way) -- the returned base says which."""
    want = list(range(kp)) if wanted is None else wanted
    if base == "merge":  # Batcher's merge, or the residue-3 split above 4 keys per list if shorter
        net = MSort(kp)
        outs = net.merge([list(range(kp // 2)), list(range(kp // 2, kp))], k=lambda n: 3 if n > 4 else 2)
        best = min((MSortProgram(kp, want, net=(net, outs)).fuse(reverse=r) for r in (True, False)),
                   key=lambda p: len(p.instrs()))
        ops = prune(NETWORKS[base](kp), want)
        other = min((Program(ops, kp, want).fuse(reverse=r) for r in (True, False)), key=lambda p: len(p.instrs()))
        return (ops, other) if len(other.instrs()) <= len(best.instrs()) else (None, best)
    if base == "msort":
        if kp not in _MSORT_NETS:
            net = MSort(kp)
            _MSORT_NETS[kp] = (net, net.sort(list(range(kp))))
        best = min((MSortProgram(kp, want, net=_MSORT_NETS[kp]).fuse(reverse=r) for r in (True, False)),
                   key=lambda p: len(p.instrs()))
        ops, other = build(tag, kp, wanted, "sort")
        if len(other.instrs()) < len(best.instrs()):
            return ops, other
        return None, best
    ops = prune(NETWORKS[base](kp), wanted if wanted is not None else range(kp))
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


NAN_CONE_TAGS = ("sort64", "sort128")  # the pair kernels' sorts (robust_pair.hip)


def emit_fused():
    lines = HEADER + [
        "// Lowered to one instruction per computed value: P2P_LO / P2P_HI (two inputs; P2P_HIS also gets the",
        "// sibling min of the same operands), P2P_LO3 / P2P_HI3 / P2P_MED3 (three inputs) -- defined by the",
        "// includer in terms of ASC (robust_nets.h).  Inputs are read from v, results written back at the end.",
        "#pragma once", ""]
    for tag, kp, wanted, base in network_specs():
        ops, prog = build(tag, kp, wanted, base)
        ins = prog.instrs()
        cnt = {k: sum(1 for _, op, _ in ins if op == k) for k in ("lo3", "hi3", "med3")}
        rng = 'all' if wanted is None else f'{wanted[0]}..{wanted[-1]}'
        if ops is None:
            shape = "three-list merge sort" if base == "msort" else "residue-3 merge"
        else:
            nce = sum(1 for o, _ in ops if o[0] == "CE") + 5 * sum(1 for o, _ in ops if o[0] == "SORT4")
            shape = (f"comparators={nce} two-input valu="
                     f"{2 * nce + sum(1 for o, _ in ops if o[0] in ('MIN', 'MAX'))} ->")
        lines.append(f"// {tag}: KP={kp} wanted={rng} {shape} {len(ins)}"
                     f" (min3 {cnt['lo3']}, max3 {cnt['hi3']}, med3 {cnt['med3']})")
        lines.append("template <bool ASC, typename T, typename H = NoHook>  // ASC=false sorts descending")
        lines.append(f"__device__ __forceinline__ void net_{tag}(T (&v)[{kp}], H&& hook = H{{}}) {{")

        def ref(n):
            return f"v[{n}]" if n < kp else f"n{n}"

        # The pair kernels' float paths test for NaN on output rank 0 alone:
        # every instruction in its cone is a min (checked here), and emitted
        # as the NaN-propagating form (P2P_LON / P2P_LO3N: v_minimum3_f32 on
        # floats, the plain min on keys), so a NaN anywhere among the inputs
        # reaches v[0] -- one compare where a packed-FMA chain over the loads
        # took ~N/4 instructions.  NaN-free inputs: the same bits.
        nan_cone = set()
        if tag in NAN_CONE_TAGS:
            byid = {i: (op, a) for i, op, a in ins}
            stack = [prog.out[0]]
            while stack:
                n = stack.pop()
                if n < kp or n in nan_cone:
                    continue
                assert byid[n][0] in ("lo", "lo3"), (tag, "rank-0 cone holds a non-min", n, byid[n][0])
                nan_cone.add(n)
                stack.extend(x for x in byid[n][1] if x is not None)
            lines.append(f"  // rank-0 cone: {len(nan_cone)} NaN-propagating mins")

        seen = set()
        for i, op, a in ins:
            # hook(v, blk) runs before the first instruction that reads input
            # block blk (16 keys) -- v still holds the inputs there
            blks = {x // 16 for x in a if x is not None and x < kp}
            for blk in sorted(blks - seen) if kp >= 16 and base in ("sort", "msort") else ():
                lines.append(f"  hook(v, {blk});")
                seen.add(blk)
            if op == "lo":
                rhs = f"P2P_LO{'N' if i in nan_cone else ''}({ref(a[0])}, {ref(a[1])})"
            elif op == "lo3" and i in nan_cone:
                rhs = f"P2P_LO3N({ref(a[0])}, {ref(a[1])}, {ref(a[2])})"
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
        for vals in inputs[:: max(1, len(inputs) // 300)].tolist() if ops is not None else ():
            got, srt = apply(ops, vals), sorted(vals)  # the classic form, spot-checked
            assert all(got[r] == srt[r] for r in want), (tag, "classic", vals)
        form = f"{len(ops)} comparators" if ops is not None else f"SSA {base}"
        print(f"{tag}: ok ({form}, {len(prog.instrs())} instructions, {len(inputs)} inputs)")


if __name__ == "__main__":
    if "--check" in sys.argv:
        check()
    elif "--search" in sys.argv:
        search_tree()
    else:
        lines = emit_classic() if "--classic" in sys.argv else emit_fused()
        with open(os.path.join(HERE, "networks.inc"), "w") as f:
            f.write("\n".join(lines))
