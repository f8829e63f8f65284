#!/usr/bin/env python3
"""Same-process A/B of the product library against other builds (round 6).

Bench-level A/Bs that alternate processes carried an order effect on these
boxes: whichever build ran first in a round read 2-3% faster, whatever it was
(profiles/r06/queue_ab/README.md).  Here every build is loaded into ONE
process (ctypes, the same ABI), the same device buffers are reduced by each
in turn, rep by rep, each launch queued behind a spin kernel and timed with
HIP events; the builds' outputs are bit-compared.  Flat FedAvg
(p2p_aggregate_f32), one launch per case -- the cfg3 plane shapes and others
-- and ("sd:K:scale") a state_dict of separately allocated tensors on the
chunk list (p2p_fedavg_split_chunks_f32, tables built once by the product).
Measurement tool, not product.
and ("rows:K:scale") the same model landed in a DeviceInbox slab (the rows
kernel).
and ("delta:n") the trainer delta over n parameters.
usage: python tools/lib_pair_ab.py <reps> <tag> [<tag> ...] -- <K:n[:median|trimmed] | sd:K:scale[:place] | rows:K:scale | rowsclone:K:scale[:carve] | delta:n> ...
  tag "prod" = p2pdl_amd/libp2pdl_hip.so, tag X = tools/libp2pdl_X.so"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from p2pdl_amd import _native as N  # noqa: E402
from p2pdl_amd import ops  # noqa: E402


def load(tag):
    path = N.LIB_PATH if tag == "prod" else os.path.join(REPO, "tools", f"libp2pdl_{tag}.so")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    f = lib.p2p_aggregate_f32
    f.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    f.restype = ctypes.c_int32
    c = lib.p2p_fedavg_split_chunks_f32
    c.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
                  ctypes.c_void_p]
    c.restype = ctypes.c_int32
    r = lib.p2p_fedavg_split_rows_f32
    r.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32, ctypes.c_float,
                  ctypes.c_void_p]
    r.restype = ctypes.c_int32
    d = lib.p2p_delta_snapshot_f32
    d.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]
    d.restype = ctypes.c_int32
    return f, c, r, d


def delta_case(fns, tags, n, reps, dev):
    """The trainer delta (p2p_delta_snapshot_f32) over n parameters: each
    build from the same cur / prev, outputs bit-compared, then timed launch by
    launch (16 B per parameter: read cur and prev, write delta and prev)."""
    cur = torch.empty(n, dtype=torch.float32, device=dev)
    prev0 = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fill_synthetic_(cur, 0x5EED0003, 1, 1e-1)
    ops.fill_synthetic_(prev0, 0x5EED0003, 2, 1e-1)
    prev, delta = prev0.clone(), torch.empty_like(cur)
    st = torch.cuda.current_stream(dev).cuda_stream
    outs = {}
    for t in tags:
        prev.copy_(prev0)
        assert fns[t][3](cur.data_ptr(), prev.data_ptr(), delta.data_ptr(), n, 0, st) == 0
        torch.cuda.synchronize()
        outs[t] = (delta.cpu().numpy().view(np.uint32), prev.cpu().numpy().view(np.uint32))
    same = all(np.array_equal(outs[t][0], outs[tags[0]][0]) and np.array_equal(outs[t][1], outs[tags[0]][1])
               for t in tags)
    ms = {t: [] for t in tags}
    for r in range(reps):
        for t in (tags if r % 2 == 0 else tags[::-1]):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(2_000_000)
            e0.record()
            fns[t][3](cur.data_ptr(), prev.data_ptr(), delta.data_ptr(), n, 0, st)
            e1.record()
            torch.cuda.synchronize()
            ms[t].append(e0.elapsed_time(e1))
    report("delta (16 B per parameter)", 2, n, same, ms)  # 4 n (K + 2) with K = 2: 16 B per parameter
    del cur, prev0, prev, delta
    torch.cuda.empty_cache()
    return same


def rows_case(fns, tags, K, scale, reps, dev):
    """ResNet-18's shapes x scale landed in a DeviceInbox slab x K: the rows
    kernel's row table and chunk table built once by the product's host code
    (ops.aggregate_slab_rows_), then every build's rows kernel over them."""
    import bench
    from p2pdl_amd.node.inbox import DeviceInbox

    sizes = [int(np.prod(sh)) for _, sh in bench.resnet18_param_shapes()] * scale
    w0 = [torch.empty(m, dtype=torch.float32, device=dev) for m in sizes]
    for l, w in enumerate(w0):
        ops.fill_synthetic_(w, 0x5EED0001 + l, 0xFFFFF, 5e-2)
    inbox = DeviceInbox({f"k{l}": w for l, w in enumerate(w0)}, k_max=K, device=dev)
    for p in range(K):
        ops.fill_synthetic_(inbox.slab[p], 0x5EED0001, p, 1e-2)
    offs = [inbox.layout[f"k{l}"][0] for l in range(len(sizes))]
    ws = [w.clone() for w in w0]
    ops._TABLES.clear()
    entry = ops.aggregate_slab_rows_(ws, inbox.slab, list(range(K)), offs, "fedavg")
    assert entry[5][0] == "rows"
    _, ch_off, ntiles = entry[5]
    base = entry[0].data_ptr()
    st = torch.cuda.current_stream(dev).cuda_stream
    outs = {}
    for t in tags:
        for w, a in zip(ws, w0):
            w.copy_(a)
        assert fns[t][2](base, K, ntiles, base + ch_off, 0, 0.1, st) == 0
        torch.cuda.synchronize()
        outs[t] = torch.cat(ws).cpu().numpy().view(np.uint32)
    same = all(np.array_equal(outs[t], outs[tags[0]]) for t in tags)
    ms = {t: [] for t in tags}
    for r in range(reps):
        for t in (tags if r % 2 == 0 else tags[::-1]):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(2_000_000)
            e0.record()
            fns[t][2](base, K, ntiles, base + ch_off, 0, 0.1, st)
            e1.record()
            torch.cuda.synchronize()
            ms[t].append(e0.elapsed_time(e1))
    report(f"rows K={K} x{scale} (DeviceInbox slab rows, {ntiles} tiles)", K, sum(sizes), same, ms)
    del inbox, ws, w0
    ops._TABLES.clear()
    torch.cuda.empty_cache()
    return same


def rows_vs_clones_case(fns, tags, K, scale, reps, dev, carve=""):
    """The bench's cfg2_dropin setup in one process (round 6): a DeviceInbox
    slab, then plain dicts of .clone()d slab-row slices (bench.py: the
    general path's pickle.loads stand-ins), and three launches alternated rep
    by rep with the first build: the rows kernel over the slab, the chunk list
    over the clones, the chunk list over the slab rows' own views.  "carve":
    a 16 GB block allocated and freed first, so the clones are carved from
    the caching allocator's cached block as after bench's cfg3 planes."""
    import bench
    from p2pdl_amd.node.inbox import DeviceInbox

    sizes = [int(np.prod(sh)) for _, sh in bench.resnet18_param_shapes()] * scale
    w0 = [torch.empty(m, dtype=torch.float32, device=dev) for m in sizes]
    for l, w in enumerate(w0):
        ops.fill_synthetic_(w, 0x5EED0001 + l, 0xFFFFF, 5e-2)
    inbox = DeviceInbox({f"k{l}": w for l, w in enumerate(w0)}, k_max=K, device=dev)
    for p in range(K):
        ops.fill_synthetic_(inbox.slab[p], 0x5EED0001, p, 1e-2)
    offs = [inbox.layout[f"k{l}"][0] for l in range(len(sizes))]
    views = [[inbox.slab[j, o:o + m] for o, m in zip(offs, sizes)] for j in range(K)]
    if carve:
        big = torch.empty(4 << 30, dtype=torch.float32, device=dev)
        del big  # cached, not returned: the clones below are split from it
    clones = [[v.clone() for v in row] for row in views]
    ws = [w.clone() for w in w0]
    st = torch.cuda.current_stream(dev).cuda_stream
    ops._TABLES.clear()
    rows = ops.aggregate_slab_rows_(ws, inbox.slab, list(range(K)), offs, "fedavg")
    _, ch_off, ntiles = rows[5]
    launches = {}
    chunk_tables = {}
    for name, src in (("chunks (clones)", clones), ("chunks (slab views)", views)):
        ptrs = np.array([[src[j][l].data_ptr() for j in range(K)] for l in range(len(sizes))], dtype=np.uint64)
        ops.aggregate_ptr_table_(ws, ptrs, "fedavg")
        e = next(reversed(ops._TABLES.values()))
        lst_off, S, segs_off, how = e[5][2]
        assert how == "chunks" and e[1] == 0
        chunk_tables[name] = (e, lst_off, S, segs_off)
    same = True
    for ti, t in enumerate(tags):
        f = fns[t]
        pre = f"{t} " if len(tags) > 1 else ""
        launches[pre + "rows (slab)"] = (lambda f=f: f[2](rows[0].data_ptr(), K, ntiles, rows[0].data_ptr() + ch_off,
                                                           0, 0.1, st))
        for name, (e, lst_off, S, segs_off) in chunk_tables.items():
            b = e[0].data_ptr()
            launches[pre + name] = (lambda f=f, b=b, lst_off=lst_off, S=S, segs_off=segs_off:
                                    f[1](b + lst_off, S, b + segs_off, K, 0, 0.1, st))
        for w, a in zip(ws, w0):  # every build's chunk list over the clones from the same w: bit-compared
            w.copy_(a)
        launches[pre + "chunks (clones)"]()
        torch.cuda.synchronize()
        got = torch.cat(ws).cpu().numpy().view(np.uint32)
        if ti == 0:
            first = got
        else:
            same &= bool(np.array_equal(got, first))
    torch.cuda.synchronize()
    names = list(launches)
    ms = {nm: [] for nm in names}
    for r in range(reps):
        for nm in (names if r % 2 == 0 else names[::-1]):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(2_000_000)
            e0.record()
            launches[nm]()
            e1.record()
            torch.cuda.synchronize()
            ms[nm].append(e0.elapsed_time(e1))
    report(f"rows vs clones K={K} x{scale} ({ntiles} tiles, builds {'/'.join(tags)}{', clones carved' if carve else ''})",
           K, sum(sizes), same, ms)
    del inbox, ws, w0, clones, views
    ops._TABLES.clear()
    torch.cuda.empty_cache()
    return same


def state_dict_case(fns, tags, K, scale, reps, dev, place="alloc"):
    """ResNet-18's 62 shapes x scale as separately allocated tensors x K: the
    chunk list and segment table built once by the product's host code
    (ops.aggregate_ptr_table_, the model tensors `ws` it points at kept),
    then every build's chunk kernel over the same tables.  `place`: "alloc"
    one allocation per tensor; "packedA" the K x L tensors packed peer-major
    in one buffer, each rounded up to A bytes (A = 512: how the caching
    allocator carves a large freed block); "offB" one allocation per tensor,
    the view starting B bytes in."""
    import bench

    sizes = [int(np.prod(sh)) for _, sh in bench.resnet18_param_shapes()] * scale
    if place.startswith("packed"):
        a = int(place[6:]) // 4
        rs = [-(-m // a) * a for m in sizes]
        buf = torch.empty(K * sum(rs), dtype=torch.float32, device=dev)
        offs = np.concatenate([[0], np.cumsum(rs)[:-1]]).astype(np.int64)
        peers = [[buf[p * sum(rs) + int(o):p * sum(rs) + int(o) + m] for o, m in zip(offs, sizes)] for p in range(K)]
    elif place.startswith("off"):
        b = int(place[3:]) // 4
        peers = [[torch.empty(m + b, dtype=torch.float32, device=dev)[b:] for m in sizes] for _ in range(K)]
    else:
        peers = [[torch.empty(m, dtype=torch.float32, device=dev) for m in sizes] for _ in range(K)]
    for p in range(K):
        for l, t in enumerate(peers[p]):
            ops.fill_synthetic_(t, 0x5EED0001 + l, p, 1e-2)
    w0 = [torch.empty(m, dtype=torch.float32, device=dev) for m in sizes]
    for l, w in enumerate(w0):
        ops.fill_synthetic_(w, 0x5EED0001 + l, 0xFFFFF, 5e-2)
    ptrs = np.array([[peers[p][l].data_ptr() for p in range(K)] for l in range(len(sizes))], dtype=np.uint64)
    ws = [w.clone() for w in w0]
    ops._TABLES.clear()
    ops.aggregate_ptr_table_(ws, ptrs, "fedavg")
    entry = next(reversed(ops._TABLES.values()))
    lst_off, S, segs_off, how = entry[5][2]
    assert how == "chunks" and entry[1] == 0, "every key on the chunk list"
    base = entry[0].data_ptr()
    st = torch.cuda.current_stream(dev).cuda_stream
    outs = {}
    for t in tags:
        for w, a in zip(ws, w0):
            w.copy_(a)
        assert fns[t][1](base + lst_off, S, base + segs_off, K, 0, 0.1, st) == 0
        torch.cuda.synchronize()
        outs[t] = torch.cat(ws).cpu().numpy().view(np.uint32)
    same = all(np.array_equal(outs[t], outs[tags[0]]) for t in tags)
    ms = {t: [] for t in tags}
    for r in range(reps):
        for t in (tags if r % 2 == 0 else tags[::-1]):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(2_000_000)
            e0.record()
            fns[t][1](base + lst_off, S, base + segs_off, K, 0, 0.1, st)
            e1.record()
            torch.cuda.synchronize()
            ms[t].append(e0.elapsed_time(e1))
    report(f"state_dict K={K} x{scale} ({len(sizes)} tensors, {place}, chunk list)", K, sum(sizes), same, ms)
    del peers, ws, w0
    ops._TABLES.clear()
    torch.cuda.empty_cache()
    return same


def report(title, K, n, same, ms):
    alg = 4.0 * n * (K + 2)
    print(f"{title} n={n:,}  bit-identical across builds: {same}")
    for t, v in ms.items():
        v = sorted(v)
        med = v[len(v) // 2]
        print(f"  {t:10s} median {med:.4f} ms  {alg / med / 1e6 / 8000:.4f} of 8 TB/s  best {alg / v[0] / 1e6 / 8000:.4f}"
              f"  worst {alg / v[-1] / 1e6 / 8000:.4f}", flush=True)


def main():
    i = sys.argv.index("--")
    reps, tags = int(sys.argv[1]), sys.argv[2:i]
    cases = [c.split(":") for c in sys.argv[i + 1:]]  # "K:n" flat, "sd:K:scale" a chunk-list state_dict
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    fns = {t: load(t) for t in tags}
    ok = True
    for case in cases:
        if case[0] == "delta":
            ok &= delta_case(fns, tags, int(case[1]), reps, dev)
            continue
        if case[0] == "rowsclone":
            ok &= rows_vs_clones_case(fns, tags, int(case[1]), int(case[2]), reps, dev, *case[3:])
            continue
        if case[0] in ("sd", "rows"):
            fn = state_dict_case if case[0] == "sd" else rows_case
            ok &= fn(fns, tags, int(case[1]), int(case[2]), reps, dev, *case[3:])
            continue
        K, n = int(case[0]), int(case[1])
        rule = {"fedavg": 0, "median": 1, "trimmed": 2}[case[2] if len(case) > 2 else "fedavg"]
        tb = ops.trim_count(K, 0.2) if rule == 2 else 0
        pitch = -(-n // 64) * 64
        slab = torch.empty((K, pitch), dtype=torch.float32, device=dev)
        for p in range(K):
            ops.fill_synthetic_(slab[p, :n], 0x5EED0002, p, 1e-2)
        table = ops.pointer_table([slab[p, :n] for p in range(K)], dev)
        w0 = torch.empty(n, dtype=torch.float32, device=dev)
        ops.fill_synthetic_(w0, 0x5EED0002, 0xFFFFF, 5e-2)
        outs = {}
        st = torch.cuda.current_stream(dev).cuda_stream
        for t, f in fns.items():
            w = w0.clone()
            assert f[0](table.data_ptr(), K, n, rule, tb, 0.1, w.data_ptr(), None, st) == 0
            torch.cuda.synchronize()
            outs[t] = w.cpu().numpy().view(np.uint32)
        same = all(np.array_equal(outs[t], outs[tags[0]]) for t in tags)
        ok &= same
        w = w0.clone()
        ms = {t: [] for t in tags}
        for r in range(reps):
            order = tags if r % 2 == 0 else tags[::-1]
            for t in order:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda._sleep(2_000_000)
                e0.record()
                fns[t][0](table.data_ptr(), K, n, rule, tb, 0.1, w.data_ptr(), None, st)
                e1.record()
                torch.cuda.synchronize()
                ms[t].append(e0.elapsed_time(e1))
        report(f"flat K={K}" + (f" {case[2]}" if len(case) > 2 else ""), K, n, same, ms)
        del slab, table, w0, w
        torch.cuda.empty_cache()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
