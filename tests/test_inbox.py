"""Receive / deserialize path: p2pdl_amd.node.inbox.

CPU tests pin the restricted parser to pickle.loads on torch-produced
pickles of the reference's message shapes (node/node.py:285 pickles a
state_dict of the models/model.py MLP); GPU tests land updates in the device
slab and aggregate them through the drop-in."""
import collections
import io
import os
import pickle
import socket
import threading
import types

import numpy as np
import pytest
import torch

import oracle
from helpers import assert_bits_equal
from p2pdl_amd.node.inbox import DeviceInbox, ZeroCopyParser, recv_message

MLP_SHAPES = [("fc1.weight", (512, 784)), ("fc1.bias", (512,)), ("fc2.weight", (256, 512)),
              ("fc2.bias", (256,)), ("fc3.weight", (10, 256)), ("fc3.bias", (10,))]  # models/model.py:6-8


def mlp_update(seed):
    out = {}
    for i, (k, s) in enumerate(MLP_SHAPES):
        out[k] = torch.from_numpy(oracle.synth(int(np.prod(s)), seed, i, 1e-2).reshape(s))
    return out


def same(raw, ref):
    assert list(raw) == list(ref)
    for k in ref:
        a = np.ascontiguousarray(raw[k].array()).reshape(-1)
        r = ref[k].contiguous().numpy().reshape(-1)
        assert raw[k].size == tuple(ref[k].shape), k
        assert a.dtype == r.dtype and np.array_equal(a.view(np.uint8), r.view(np.uint8)), k


# the Python machine and its C++ port (csrc/wire.cpp) on every case
PARSERS = [lambda d: ZeroCopyParser(d, native=False).parse(), lambda d: ZeroCopyParser(d, native=True).parse()]


@pytest.mark.parametrize("parse", PARSERS, ids=["python", "native"])
def test_parser_matches_pickle_loads_mlp_update(parse):
    upd = mlp_update(1)
    data = pickle.dumps(upd)  # reference node/node.py:285
    same(parse(data), pickle.loads(data))


@pytest.mark.parametrize("proto", [3, 4, 5])
@pytest.mark.parametrize("parse", PARSERS, ids=["python", "native"])
def test_parser_batchnorm_scalars_views_and_ordereddict(parse, proto):
    net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.BatchNorm1d(5))
    sd = net.state_dict()  # OrderedDict incl. an int64 0-d buffer
    sd["view.t"] = torch.arange(12, dtype=torch.float32).reshape(3, 4).t()  # strided view
    sd["view.slice"] = torch.arange(20, dtype=torch.float32)[5:9]           # storage offset
    sd["x" * 300] = torch.ones(3)                                           # BINUNICODE key
    data = pickle.dumps(sd, protocol=proto)
    same(parse(data), pickle.loads(data))


def test_native_parser_is_the_default():
    """The receive path runs the C++ machine (csrc/wire.cpp) when it is built
    -- __graft_entry__.build() builds it beside the HIP library."""
    from p2pdl_amd import _wire  # noqa: F401

    assert ZeroCopyParser(b"").native is True


def test_zero_copy_parser_payloads_alias_the_message():
    data = bytearray(pickle.dumps({"w": torch.arange(1000, dtype=torch.float32)}))
    raw = ZeroCopyParser(data).parse()
    arr = raw["w"].array()
    assert arr[7] == 7.0
    i = bytes(data).index(np.arange(1000, dtype=np.float32)[5:9].tobytes())
    data[i:i + 4] = np.float32(-1).tobytes()  # mutate the message: the view sees it
    assert raw["w"].array()[5] == -1.0


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


@pytest.mark.parametrize("payload", [
    {"a": _Evil()},
    {"a": torch.ones(2), "b": _Evil()},
    [torch.ones(3)],                       # not a dict of tensors
    {"a": 3},
])
def test_parser_rejects_anything_but_tensors(payload):
    for parse in PARSERS:
        with pytest.raises(pickle.UnpicklingError):
            parse(pickle.dumps(payload))


def test_zero_copy_parser_rejects_protocol_2_and_truncation():
    with pytest.raises(pickle.UnpicklingError):
        ZeroCopyParser(pickle.dumps({"a": torch.ones(2)}, protocol=2)).parse()
    data = pickle.dumps({"a": torch.ones(2)})
    for cut in range(1, len(data)):  # every truncation: UnpicklingError and nothing else
        for parse in PARSERS:
            with pytest.raises(pickle.UnpicklingError):
                parse(data[:cut])


def test_parsers_raise_only_unpickling_error_on_corrupted_bytes():
    """A listener catching pickle.UnpicklingError must survive any peer bytes
    (KeyError / IndexError / struct.error used to escape)."""
    rng = np.random.default_rng(0)
    data = pickle.dumps(torch.nn.Sequential(torch.nn.Linear(3, 2), torch.nn.BatchNorm1d(2)).state_dict())
    for _ in range(3000):
        m = bytearray(data)
        for i in rng.integers(0, len(m), rng.integers(1, 4)):
            m[i] = int(rng.integers(0, 256))
        for parse in PARSERS:
            try:
                parse(bytes(m))
            except pickle.UnpicklingError:
                pass


def test_native_and_python_machines_agree_on_corrupted_bytes():
    """Differential fuzz of the two machines: on every corruption both reject,
    or both accept with the same keys, dtypes, views and payload bytes."""
    rng = np.random.default_rng(7)
    data = pickle.dumps(torch.nn.Sequential(torch.nn.Linear(3, 2), torch.nn.BatchNorm1d(2)).state_dict())

    def run(native, d):
        try:
            r = ZeroCopyParser(d, native=native).parse()
        except pickle.UnpicklingError:
            return None
        return [(k, v.storage.dtype, v.storage.numel, v.storage.location, v.offset, v.size, v.stride,
                 bytes(v.storage.data)) for k, v in r.items()]

    accepted = 0
    for _ in range(3000):
        m = bytearray(data)
        for i in rng.integers(0, len(m), rng.integers(1, 4)):
            m[i] = int(rng.integers(0, 256))
        a, b = run(False, bytes(m)), run(True, bytes(m))
        assert a == b, bytes(m)
        accepted += a is not None
    assert accepted > 0  # some corruptions hit payload bytes only


# ---- forged updates: the storage blob and the tensor view come from the peer
def _good_blob(n=2):
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        fn, (blob,) = torch.ones(n).storage().__reduce__()  # what torch pickles per tensor
    assert fn is torch.storage._load_from_bytes
    return blob


class _Storage:
    def __init__(self, blob):
        self.blob = blob

    def __reduce__(self):
        return (torch.storage._load_from_bytes, (self.blob,))


class _Tensor:
    def __init__(self, blob, offset=0, size=(2,), stride=(1,)):
        self.args = (_Storage(blob), offset, size, stride, False, collections.OrderedDict())

    def __reduce__(self):
        return (torch._utils._rebuild_tensor_v2, self.args)


def _forged(blob, **view):
    return pickle.dumps({"a": _Tensor(blob, **view)})


def test_forged_update_with_honest_view_parses():
    data = _forged(_good_blob(4), offset=1, size=(3,), stride=(1,))
    for parse in PARSERS:
        raw = parse(data)
        assert raw["a"].array().tolist() == [1.0, 1.0, 1.0]


@pytest.mark.parametrize("which", [0, 1, 2])
def test_storage_header_pickles_cannot_run_code(which, tmp_path):
    """the magic / protocol-version / sys_info pickles of
    the storage blob went through a plain pickle.Unpickler.  A GLOBAL/REDUCE
    nested in any of them must be refused, and must not run."""
    blob = _good_blob()
    f = io.BytesIO(blob)
    starts = [0]
    for _ in range(3):  # the three header pickles precede the storage record
        pickle.Unpickler(f).load()  # our own, honest blob
        starts.append(f.tell())
    marker = tmp_path / "pwned"
    evil = pickle.dumps(_Touch(str(marker)))
    forged = blob[:starts[which]] + evil + blob[starts[which + 1]:]
    for parse in PARSERS:
        with pytest.raises(pickle.UnpicklingError):
            parse(_forged(forged))
    assert not marker.exists()


class _Touch:
    def __init__(self, path):
        self.path = path

    def __reduce__(self):
        return (open, (self.path, "w"))


@pytest.mark.parametrize("view", [
    dict(size=(1000,)),                       # more elements than the storage holds
    dict(offset=5, size=(1,)),                # offset past the end
    dict(offset=1, size=(2,)),                # last element one past the end
    dict(size=(2, 2), stride=(1, 1)),         # strided view reaching element 2
    dict(size=(2,), stride=(-1,)),            # negative stride
    dict(offset=-1, size=(1,)),               # negative offset
    dict(size=(2,), stride=(1, 1)),           # rank mismatch
    dict(size=(2.0,)),                        # non-integer size
])
def test_out_of_bounds_tensor_views_are_refused(view):
    """a peer claiming a view larger than its storage made
    as_strided read host memory past the message."""
    data = _forged(_good_blob(2), **view)
    for parse in PARSERS:
        with pytest.raises(pickle.UnpicklingError):
            parse(data)


@pytest.mark.parametrize("view", [
    dict(size=(2 ** 33,), stride=(0,)),       # 8 G elements over one storage element
    dict(size=(2, 3), stride=(0, 1)),         # a repeated row
    dict(size=(3, 3), stride=(1, 1)),         # overlapping rows, 9 elements over 5
])
def test_repeating_tensor_views_are_refused(view):
    """a zero-stride / overlapping view inside its
    storage passed the bounds check, and a key outside the fp32 template was
    then copied element by element -- a few hundred bytes asking for 32 GB."""
    data = _forged(_good_blob(5), **view)
    for parse in PARSERS:
        with pytest.raises(pickle.UnpicklingError):
            parse(data)
    # dense views of every shape still parse, incl. size-1 dims with any stride
    for ok in (dict(size=(5,)), dict(size=(1, 5), stride=(0, 1)), dict(size=(5, 1), stride=(1, 0))):
        raw = ZeroCopyParser(_forged(_good_blob(5), **ok)).parse()
        assert raw["a"].array().size == 5


def test_many_marks_parse_in_linear_time():
    """closing a MARK copied the rest of the stack (O(n^2) in a
    listener thread for a message of MARK ... TUPLE pairs)."""
    import time

    n = 200_000
    body = b"\x80\x04" + b"(" * n + b")" + b"t" * n + b"."  # PROTO 4, n MARKs, EMPTY_TUPLE, n TUPLEs
    t0 = time.perf_counter()
    with pytest.raises(pickle.UnpicklingError):  # well-formed, but not a state_dict
        ZeroCopyParser(body).parse()
    assert time.perf_counter() - t0 < 5.0


def test_build_cannot_shadow_dict_methods():
    """A pickle's BUILD on the OrderedDict may set only torch's `_metadata`."""
    class Shadow(collections.OrderedDict):
        def __reduce__(self):
            return (collections.OrderedDict, (), {"values": None}, None, iter(self.items()))

    d = Shadow()
    d["a"] = torch.ones(2)
    data = pickle.dumps(d)
    with pytest.raises(pickle.UnpicklingError):
        ZeroCopyParser(data).parse()
    raw = ZeroCopyParser(pickle.dumps(torch.nn.Linear(2, 2).state_dict())).parse()
    assert type(raw) is collections.OrderedDict and not raw.__dict__  # a fresh dict


def test_huge_memo_index_is_cheap():
    """A LONG_BINPUT with a ~1.5e9 index made the C unpickler allocate a
    12 GB memo array (found by the corruption fuzz above); the machine's
    memo is a dict."""
    import time

    data = bytearray(pickle.dumps({"b": torch.ones(2)}))
    i = data.index(b"\x94", data.index(b"_rebuild_tensor_v2"))  # a MEMOIZE after the global
    data[i:i + 1] = b"r\xff\xff\xff\x5f"  # LONG_BINPUT 0x5fffffff
    t0 = time.perf_counter()
    try:
        ZeroCopyParser(bytes(data)).parse()
    except pickle.UnpicklingError:
        pass
    assert time.perf_counter() - t0 < 1.0


@pytest.mark.parametrize("length", [2 ** 63 - 1, 2 ** 63 - 9, 2 ** 63 - 4096, 2 ** 64 - 1, 2 ** 62])
def test_binbytes8_huge_length_is_refused(length):
    """a BINBYTES8 length near INT64_MAX overflowed the
    C++ machine's bounds check (p + k wrapped negative) and sent the parser
    past the message.  Both machines must refuse it as a truncated pickle."""
    body = b"\x80\x05\x95\x00\x00\x00\x00\x00\x00\x00\x00}\x94\x8c\x01a\x94\x8e" + length.to_bytes(8, "little")
    for data in (body + b"xyz.", body):
        for parse in PARSERS:
            with pytest.raises(pickle.UnpicklingError):
                parse(data)


@pytest.mark.parametrize("parse", PARSERS, ids=["python", "native"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_parser_16bit_storages(parse, dtype):
    """BFloat16Storage payloads parse (held as uint16 bit
    patterns) and materialise as the torch dtype, bit-equal to pickle.loads."""
    g = torch.Generator().manual_seed(3)
    sd = collections.OrderedDict(w=torch.randn(33, 7, generator=g).to(dtype), b=torch.randn(5, generator=g).to(dtype))
    sd["t"] = sd["w"].t()  # a strided view of the same storage
    data = pickle.dumps(sd)
    raw = parse(data)
    ref = pickle.loads(data)
    assert list(raw) == list(ref)
    for key in ref:
        got = raw[key].tensor("cpu")
        assert got.dtype == dtype and got.shape == ref[key].shape, key
        assert torch.equal(got.view(torch.int16), ref[key].contiguous().view(torch.int16)), key


def test_recv_message_framing_and_early_close():
    a, b = socket.socketpair()
    msg = pickle.dumps({"type": "model_update", "model": pickle.dumps(mlp_update(2)), "addr": "x", "port": 1})

    def send():
        b.sendall(len(msg).to_bytes(4, "big"))
        for i in range(0, len(msg), 4096):  # the reference's 4 KiB pieces
            b.sendall(msg[i:i + 4096])
        b.sendall((1000).to_bytes(4, "big") + b"short")  # a truncated second message
        b.close()

    th = threading.Thread(target=send)
    th.start()
    got = recv_message(a)
    assert bytes(got) == msg
    assert recv_message(a) is None  # peer closed early: dropped, like node/node.py:111
    th.join()
    a.close()


@pytest.mark.gpu
def test_device_inbox_lands_bit_exact_and_aggregates(cuda, monkeypatch):
    from p2pdl_amd.aggregator import aggregation as agg

    monkeypatch.setattr(agg, "broadcast_global_model_update", lambda self: None)
    k = 5
    template = {name: torch.zeros(s, device=cuda) for name, s in MLP_SHAPES}
    inbox = DeviceInbox(template, k_max=8, device=cuda)
    ser = [pickle.dumps(mlp_update(10 + j)) for j in range(k)]
    landed = [inbox.land(s) for s in ser]
    torch.cuda.synchronize()
    for s, got in zip(ser, landed):
        ref = pickle.loads(s)
        assert list(got) == list(ref)
        for key in ref:
            assert got[key].is_cuda and got[key].shape == ref[key].shape
            assert_bits_equal(got[key].cpu().numpy(), ref[key].numpy(), what=key)
    # the landed views feed the drop-in unchanged (node/node.py:138 -> :316)
    n = sum(int(np.prod(s)) for _, s in MLP_SHAPES)
    w = oracle.synth(n, 3, 0xFFFFF, 5e-2)
    model = torch.nn.Module()
    offs = 0
    for name, s in MLP_SHAPES:
        m = int(np.prod(s))
        mod, attr = name.split(".")
        if not hasattr(model, mod):
            model.add_module(mod, torch.nn.Module())
        getattr(model, mod).register_parameter(attr, torch.nn.Parameter(
            torch.from_numpy(w[offs:offs + m].reshape(s).copy()).to(cuda)))
        offs += m
    node = types.SimpleNamespace(model=model, trainers_list=[0] * k, addr="a", port=1, neighbors=[],
                                 received_models=[{"model": u, "sender": j} for j, u in enumerate(landed)])
    agg.aggregate_models(node)
    got = np.concatenate([t.detach().cpu().numpy().reshape(-1) for t in model.state_dict().values()])
    flat = [np.concatenate([pickle.loads(s)[name].numpy().reshape(-1) for name, _ in MLP_SHAPES]) for s in ser]
    want, _ = oracle.fedavg(flat, w)
    assert_bits_equal(got, want, what="fedavg over landed updates")


@pytest.mark.gpu
def test_device_inbox_parses_cuda_pickles(cuda):
    upd = {k: v.to(cuda) for k, v in mlp_update(4).items()}
    data = pickle.dumps(upd)  # a CUDA sender's bytes (storage location 'cuda:0')
    inbox = DeviceInbox({k: v for k, v in upd.items()}, k_max=1, device=cuda)
    got = inbox.land(data, 0)
    torch.cuda.synchronize()
    for key in upd:
        assert torch.equal(got[key], upd[key]), key


@pytest.mark.gpu
def test_broadcast_from_gpu_model_one_transfer(cuda):
    """the GPU model's broadcast carries the same
    keys/values (bit-exact) with the reference framing."""
    import socket as sk

    from p2pdl_amd.aggregator import aggregation as agg

    net = torch.nn.Sequential(torch.nn.Linear(33, 64), torch.nn.BatchNorm1d(64), torch.nn.Linear(64, 10)).to(cuda)
    srv = sk.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    got = {}

    def serve():
        c, _ = srv.accept()
        got["msg"] = pickle.loads(bytes(recv_message(c)))
        c.close()

    th = threading.Thread(target=serve)
    th.start()
    nd = types.SimpleNamespace(model=net, addr="127.0.0.1", port=9,
                               neighbors=[types.SimpleNamespace(addr="127.0.0.1", port=srv.getsockname()[1])])
    agg.broadcast_global_model_update(nd)
    th.join(10)
    srv.close()
    msg = got["msg"]
    assert msg["type"] == "global_model_update" and msg["addr"] == "127.0.0.1" and msg["port"] == 9
    ref = net.state_dict()
    assert list(msg["model"]) == list(ref)
    for k, v in ref.items():
        assert msg["model"][k].device == v.device and torch.equal(msg["model"][k], v), k  # as the reference's pickle
        assert msg["model"][k].untyped_storage().nbytes() == v.numel() * v.element_size(), k


@pytest.mark.gpu
def test_device_inbox_concurrent_landing(cuda):
    """land() is called from one listener thread per connection
    (reference node/node.py:89); concurrent calls must take distinct rows and
    never mix two updates in a staging row."""
    k = 8
    template = {name: torch.zeros(s, device=cuda) for name, s in MLP_SHAPES}
    inbox = DeviceInbox(template, k_max=k, device=cuda)
    ser = [pickle.dumps(mlp_update(40 + j)) for j in range(k)]
    got = [None] * k
    barrier = threading.Barrier(k)

    def worker(j):
        barrier.wait()
        got[j] = inbox.land(ser[j])

    ths = [threading.Thread(target=worker, args=(j,)) for j in range(k)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(60)
    torch.cuda.synchronize()
    assert inbox.count == k
    rows = {got[j]["fc1.weight"].data_ptr() for j in range(k)}
    assert len(rows) == k  # every update in its own slab row
    for j in range(k):
        ref = pickle.loads(ser[j])
        for key in ref:
            assert_bits_equal(got[j][key].cpu().numpy(), ref[key].numpy(), what=f"update {j} {key}")


@pytest.mark.gpu
def test_device_inbox_digest_overlapped_with_landing(cuda):
    """land(..., digest=True) hashes the serialized update --
    the bytes the tester signs in its echo (node/node.py:144, crypto.py:54-57)
    -- beside the parse / copy / DMA; digests equal hashlib's, concurrent
    landings keep row <-> digest pairs, rows without digest refuse."""
    import hashlib

    k = 6
    template = {name: torch.zeros(s, device=cuda) for name, s in MLP_SHAPES}
    inbox = DeviceInbox(template, k_max=k + 1, device=cuda)
    for key, (off, _, _) in inbox.layout.items():
        assert off % 64 == 0, key  # 256-B aligned tensor views
    ser = [pickle.dumps(mlp_update(70 + j)) for j in range(k)]
    got = [None] * k
    barrier = threading.Barrier(k)

    def worker(j):
        barrier.wait()
        got[j] = inbox.land(ser[j], j, digest=True)

    ths = [threading.Thread(target=worker, args=(j,)) for j in range(k)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(60)
    for j in range(k):
        assert inbox.digest(j) == hashlib.sha256(ser[j]).digest(), j
        assert got[j].row == j
    inbox.land(ser[0], k)
    with pytest.raises(KeyError):
        inbox.digest(k)
    inbox.land(ser[1], 0)  # re-landed without a digest, row 0's old one is gone
    with pytest.raises(KeyError):
        inbox.digest(0)
    inbox.reset()
    with pytest.raises(KeyError):
        inbox.digest(0)


@pytest.mark.gpu
@pytest.mark.parametrize("rule", ["fedavg", "median", "trimmed", "fedavg_torch_gpu"])
def test_landed_updates_take_the_slab_fast_path(cuda, rule, monkeypatch):
    """aggregate_models on DeviceInbox-landed updates builds its kernel table
    from (slab, rows, key offsets) -- no per-tensor work -- and gives the same
    bits as the general path and the oracle; one plain dict among them sends
    the call down the general path."""
    from p2pdl_amd import ops
    from p2pdl_amd.aggregator import aggregation as agg

    monkeypatch.setattr(agg, "broadcast_global_model_update", lambda self: None)
    k = 7
    template = {name: torch.zeros(s, device=cuda) for name, s in MLP_SHAPES}
    inbox = DeviceInbox(template, k_max=k, device=cuda)
    ser = [pickle.dumps(mlp_update(60 + j)) for j in range(k)]
    landed = [inbox.land(s) for s in ser]
    n = sum(int(np.prod(s)) for _, s in MLP_SHAPES)
    w = oracle.synth(n, 5, 0xFFFFF, 5e-2)
    flat = [np.concatenate([pickle.loads(s)[name].numpy().reshape(-1) for name, _ in MLP_SHAPES]) for s in ser]
    if rule in ("fedavg", "fedavg_torch_gpu"):
        want, _ = oracle.fedavg(flat, w, torch_gpu=rule == "fedavg_torch_gpu")
    else:
        r = ops.rule_id(rule)
        want, _ = oracle.robust(flat, r, ops.trim_count(k) if r == 2 else 0, w=w)

    def run(updates):
        model = torch.nn.Module()
        offs = 0
        for name, s in MLP_SHAPES:
            m = int(np.prod(s))
            mod, attr = name.split(".")
            if not hasattr(model, mod):
                model.add_module(mod, torch.nn.Module())
            getattr(model, mod).register_parameter(attr, torch.nn.Parameter(
                torch.from_numpy(w[offs:offs + m].reshape(s).copy()).to(cuda)))
            offs += m
        node = types.SimpleNamespace(model=model, trainers_list=[0] * k, addr="a", port=1, neighbors=[],
                                     received_models=[{"model": u, "sender": j} for j, u in enumerate(updates)])
        agg.aggregate_models(node, rule=rule)
        assert node.received_models == []
        return np.concatenate([t.detach().cpu().numpy().reshape(-1) for t in model.state_dict().values()])

    def boom(*a, **kw):
        raise AssertionError("wrong path")

    with monkeypatch.context() as m:
        m.setattr(ops, "aggregate_segments_", boom)  # must not be reached
        assert_bits_equal(run(landed), want, what=f"fast path {rule}")
    with monkeypatch.context() as m:
        m.setattr(ops, "aggregate_slab_rows_", boom)
        mixed = landed[:-1] + [dict(landed[-1])]  # a plain dict: general path
        assert_bits_equal(run(mixed), want, what=f"general path {rule}")
    with pytest.raises(TypeError):
        landed[0]["fc1.weight"] = torch.zeros(1)
    with pytest.raises(TypeError):
        del landed[0]["fc1.bias"]
    back = pickle.loads(pickle.dumps(landed[0]))  # copies, not the slab
    assert type(back) is collections.OrderedDict and list(back) == list(landed[0])
    assert back["fc3.bias"].untyped_storage().nbytes() == 10 * 4


@pytest.mark.gpu
def test_slab_table_cache_across_rounds_and_streams(cuda, monkeypatch):
    """The fast path caches its device segment table by the addresses and
    sizes it encodes: round 2 reuses round 1's table for NEW values in the
    same slab rows (bit-exact vs the oracle both rounds), a different row set
    or model builds a new table, and a launch on another stream is correct."""
    from p2pdl_amd import ops
    from p2pdl_amd.aggregator import aggregation as agg

    monkeypatch.setattr(agg, "broadcast_global_model_update", lambda self: None)
    k = 4
    template = {name: torch.zeros(s, device=cuda) for name, s in MLP_SHAPES}
    inbox = DeviceInbox(template, k_max=k + 1, device=cuda)
    n = sum(int(np.prod(s)) for _, s in MLP_SHAPES)
    w0 = oracle.synth(n, 9, 0xFFFFF, 5e-2)
    model = torch.nn.Module()
    offs = 0
    for name, s in MLP_SHAPES:
        m = int(np.prod(s))
        mod, attr = name.split(".")
        if not hasattr(model, mod):
            model.add_module(mod, torch.nn.Module())
        getattr(model, mod).register_parameter(attr, torch.nn.Parameter(
            torch.from_numpy(w0[offs:offs + m].reshape(s).copy()).to(cuda)))
        offs += m
    node = types.SimpleNamespace(model=model, trainers_list=[0] * k, addr="a", port=1, neighbors=[],
                                 received_models=[])
    w = w0
    side = torch.cuda.Stream(cuda)
    for rnd, (rows, stream) in enumerate([(range(k), None), (range(k), None), (range(1, k + 1), None),
                                          (range(1, k + 1), torch.cuda.Stream(cuda)), (range(k), "land")]):
        inbox.reset()
        ser = [pickle.dumps(mlp_update(90 + 10 * rnd + j)) for j in range(k)]
        if stream == "land":
            # a listener thread lands on its own stream; the
            # aggregator launches on its current stream with no sync of its own
            landed = [None] * k

            def listener():
                with torch.cuda.stream(side):
                    for j, (s_, r) in enumerate(zip(ser, rows)):
                        landed[j] = inbox.land(s_, r)

            th = threading.Thread(target=listener)
            th.start()
            th.join(60)
            stream = None
        else:
            landed = [inbox.land(s_, r) for s_, r in zip(ser, rows)]
        node.received_models = [{"model": u, "sender": j} for j, u in enumerate(landed)]
        flat = [np.concatenate([pickle.loads(s)[name].numpy().reshape(-1) for name, _ in MLP_SHAPES])
                for s in ser]
        want, _ = oracle.fedavg(flat, w)
        if stream is None:
            agg.aggregate_models(node)
        else:
            stream.wait_stream(torch.cuda.current_stream(cuda))
            with torch.cuda.stream(stream):
                agg.aggregate_models(node)
            torch.cuda.current_stream(cuda).wait_stream(stream)
        got = np.concatenate([t.detach().cpu().numpy().reshape(-1) for t in model.state_dict().values()])
        assert_bits_equal(got, want, what=f"round {rnd}")
        w = want
    mine = [key for key in ops._TABLES if key[1:3] == (inbox.slab.data_ptr(), k + 1)]
    assert len(mine) == 2  # one table per row set (0..3, 1..4), reused across rounds and streams

    # the launch cache on the model-state entry: same rows + rule -> relaunch
    # (no aggregate_slab_rows_ call); a rule change on the same rows -> a new
    # table, not the FedAvg one launched again
    calls = {"relaunch": 0, "table": 0}
    real_relaunch, real_rows = ops.relaunch, ops.aggregate_slab_rows_

    def counted(name, fn):
        def f(*a, **kw):
            calls[name] += 1
            return fn(*a, **kw)
        return f

    monkeypatch.setattr(ops, "relaunch", counted("relaunch", real_relaunch))
    monkeypatch.setattr(ops, "aggregate_slab_rows_", counted("table", real_rows))
    for rnd, rule in enumerate(["fedavg", "fedavg", "median", "median", "trimmed", "fedavg"]):
        inbox.reset()
        ser = [pickle.dumps(mlp_update(300 + 10 * rnd + j)) for j in range(k)]
        landed = [inbox.land(s_, r) for s_, r in zip(ser, range(k))]
        node.received_models = [{"model": u, "sender": j} for j, u in enumerate(landed)]
        flat = [np.concatenate([pickle.loads(s)[name].numpy().reshape(-1) for name, _ in MLP_SHAPES])
                for s in ser]
        if rule == "fedavg":
            want, _ = oracle.fedavg(flat, w)
        else:
            r = ops.rule_id(rule)
            want, _ = oracle.robust(flat, r, ops.trim_count(k) if r == 2 else 0, w=w)
        agg.aggregate_models(node, rule=rule)
        got = np.concatenate([t.detach().cpu().numpy().reshape(-1) for t in model.state_dict().values()])
        assert_bits_equal(got, want, what=f"launch-cache round {rnd} {rule}")
        w = want
    # fedavg (the launch cached by the last round above), fedavg, median (new
    # table), median, trimmed (new table), fedavg (launch cache holds trimmed:
    # aggregate_slab_rows_, which finds the FedAvg table in _TABLES and
    # relaunches it)
    assert calls == {"relaunch": 4, "table": 3}


# ---- K5 device path: the message in pinned memory, one DMA, the landing kernel
def _pinned(inbox, data):
    m = inbox.message_buffer(len(data))
    m.buf[:len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    return m


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [3, 4, 5])
def test_pinned_landing_matches_pickle_loads(cuda, proto):
    """p2p_land_segments_f32 places every payload (arbitrary byte offsets in
    the pickle: the 0-d / int64 BatchNorm entries shift them) bit-exactly;
    non-fp32 entries become their own tensors as on the staging path."""
    net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.BatchNorm1d(5), torch.nn.Linear(5, 3))
    rows = []
    for j in range(4):
        torch.manual_seed(j)
        sd = {k: (v + torch.randn_like(v) if v.is_floating_point() else v + j) for k, v in net.state_dict().items()}
        sd.update({f"x{j}.w": torch.randn(1 + j, 37)})  # extra key: not in the template, small tensor
        rows.append(pickle.dumps(sd, protocol=proto))
    template = {k: v.to(cuda) for k, v in net.state_dict().items()}
    inbox = DeviceInbox(template, k_max=4, device=cuda)
    got = [inbox.land(_pinned(inbox, d)) for d in rows]
    torch.cuda.synchronize()
    for d, g in zip(rows, got):
        ref = pickle.loads(d)
        assert list(g) == list(ref)
        for key in ref:
            assert g[key].is_cuda and g[key].dtype == ref[key].dtype and g[key].shape == ref[key].shape, key
            assert torch.equal(g[key].cpu(), ref[key]), key
    assert all(set(g.slab_keys) == {k for k, v in template.items() if v.dtype == torch.float32} for g in got)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["float16", "bfloat16"])
@pytest.mark.parametrize("pinned", [False, True])
def test_16bit_model_lands_and_aggregates(cuda, dt, pinned, monkeypatch):
    """A model.half() / bfloat16 node: the 16-bit updates are not
    slab rows -- land() makes each its own device tensor of the storage's
    dtype (HalfStorage / BFloat16Storage, bits as sent) -- and
    aggregate_models over the landed updates == oracle.fedavg16_np (the
    reference's fp32-op-then-round loop, aggregation.py:15-38, pinned to its
    own CPU run by tests/golden/fedavg16_golden.npz)."""
    from p2pdl_amd.aggregator import aggregation as agg

    monkeypatch.setattr(agg, "broadcast_global_model_update", lambda self: None)
    tdt = {"float16": torch.float16, "bfloat16": torch.bfloat16}[dt]
    k, n = 3, sum(int(np.prod(s)) for _, s in MLP_SHAPES)

    def tensors(bits):
        out, o = {}, 0
        for name, s in MLP_SHAPES:
            m = int(np.prod(s))
            out[name] = torch.from_numpy(bits[o:o + m].view(np.int16).copy()).view(tdt).reshape(s)
            o += m
        return out

    w = oracle.round_16(oracle.synth_np(n, 41, 0xFFFFF, 5e-2), dt)
    peers = [oracle.round_16(oracle.synth_np(n, 41, p, 1e-2), dt) for p in range(k)]
    template = {name: t.to(cuda) for name, t in tensors(w).items()}
    inbox = DeviceInbox(template, k_max=k, device=cuda)
    assert inbox.row == 0  # no fp32 entry: no slab row
    ser = [pickle.dumps(tensors(p)) for p in peers]
    landed = [inbox.land(_pinned(inbox, s) if pinned else s) for s in ser]
    for got, p in zip(landed, peers):
        assert list(got) == [name for name, _ in MLP_SHAPES] and not got.slab_keys
        bits = np.concatenate([got[name].view(torch.int16).cpu().numpy().view(np.uint16).reshape(-1)
                               for name, _ in MLP_SHAPES])
        assert np.array_equal(bits, p) and all(got[name].dtype == tdt for name, _ in MLP_SHAPES)
    model = torch.nn.Module()
    for name, t in template.items():
        model.register_parameter(name.replace(".", "__"), torch.nn.Parameter(t.clone(), requires_grad=False))
    ups = [{name.replace(".", "__"): v for name, v in dict(u).items()} for u in landed]
    node = types.SimpleNamespace(model=model, trainers_list=[0] * k, addr="a", port=1, neighbors=[],
                                 received_models=[{"model": u, "sender": j} for j, u in enumerate(ups)])
    agg.aggregate_models(node)
    torch.cuda.synchronize()
    got = np.concatenate([t.detach().view(torch.int16).cpu().numpy().view(np.uint16).reshape(-1)
                          for t in model.state_dict().values()])
    want = oracle.fedavg16_np(peers, w, dt)
    fg, fw = oracle.to_f32_16(got, dt), oracle.to_f32_16(want, dt)
    assert np.all((got == want) | (np.isnan(fg) & np.isnan(fw))), f"{dt}: {np.count_nonzero(got != want)} differ"
    assert node.received_models == []


@pytest.mark.gpu
def test_pinned_landing_every_misalignment_and_tail(cuda):
    """Payload offsets mod 4 = 0..3 (a prefix key of 1..4 bytes of name moves
    them) and a tensor ending at the last payload byte of the message."""
    for pad in range(1, 5):
        upd = collections.OrderedDict([("p" * pad, torch.arange(3, dtype=torch.float32)),
                                       ("w", torch.randn(4099)), ("b", torch.randn(1))])
        data = pickle.dumps(upd)
        template = {k: torch.zeros_like(v, device=cuda) for k, v in upd.items()}
        inbox = DeviceInbox(template, k_max=1, device=cuda)
        got = inbox.land(_pinned(inbox, data), 0)
        torch.cuda.synchronize()
        for key, v in upd.items():
            assert_bits_equal(got[key].cpu().numpy(), v.numpy(), what=f"pad {pad} {key}")


@pytest.mark.gpu
def test_pinned_landing_resnet_sized_update_and_digest(cuda):
    """Large conv / fc payloads (2.9M params, multi-tile segments): the
    landing kernel vs pickle.loads, the overlapped digest vs hashlib, pinned
    buffers reused from the pool across rounds."""
    import hashlib

    shapes = [("conv.weight", (64, 3, 7, 7)), ("fc.weight", (1000, 512)), ("fc.bias", (1000,))] + \
        [(f"layer{i}.weight", (128, 128, 3, 3)) for i in range(4)]
    template = {k: torch.zeros(s, device=cuda) for k, s in shapes}
    inbox = DeviceInbox(template, k_max=3, device=cuda)
    for rnd in range(2):
        inbox.reset()
        ser = []
        for j in range(3):
            g = torch.Generator().manual_seed(100 * rnd + j)
            ser.append(pickle.dumps({k: torch.randn(s, generator=g) for k, s in shapes}))
        got = [inbox.land(_pinned(inbox, d), digest=True) for d in ser]
        torch.cuda.synchronize()
        for j, (d, g) in enumerate(zip(ser, got)):
            ref = pickle.loads(d)
            for key in ref:
                assert torch.equal(g[key].cpu(), ref[key]), (rnd, j, key)
            assert inbox.digest(j) == hashlib.sha256(d).digest()
    assert len(inbox._pinned_free) <= 3  # buffers come back to the pool and are reused


@pytest.mark.gpu
def test_pinned_landing_strided_view_takes_staging_path(cuda):
    """A transposed (non-dense) fp32 view cannot be a byte run: land() falls
    back to the staging copy and the values still match pickle.loads."""
    base = torch.randn(6, 4)
    upd = {"w": base.t(), "b": torch.randn(4)}
    data = pickle.dumps(upd)
    template = {"w": torch.zeros(4, 6, device=cuda), "b": torch.zeros(4, device=cuda)}
    inbox = DeviceInbox(template, k_max=1, device=cuda)
    got = inbox.land(_pinned(inbox, data), 0)
    torch.cuda.synchronize()
    assert torch.equal(got["w"].cpu(), upd["w"]) and torch.equal(got["b"].cpu(), upd["b"])


@pytest.mark.gpu
def test_inbox_recv_into_pinned_and_land(cuda):
    """DeviceInbox.recv: the reference framing (node/node.py:99-112) read into
    a pinned buffer of the inbox; early close returns None."""
    template = {name: torch.zeros(s, device=cuda) for name, s in MLP_SHAPES}
    inbox = DeviceInbox(template, k_max=2, device=cuda)
    data = pickle.dumps(mlp_update(7))
    a, b = socket.socketpair()
    th = threading.Thread(target=lambda: (a.sendall(len(data).to_bytes(4, "big") + data), a.close()))
    th.start()
    msg = inbox.recv(b)
    th.join(10)
    got = inbox.land(msg)
    torch.cuda.synchronize()
    ref = pickle.loads(data)
    for key in ref:
        assert_bits_equal(got[key].cpu().numpy(), ref[key].numpy(), what=key)
    c, d = socket.socketpair()
    c.sendall((100).to_bytes(4, "big") + b"xx")
    c.close()
    assert inbox.recv(d) is None
    b.close()
    d.close()


@pytest.mark.gpu
def test_envelope_received_pinned_lands_in_place(cuda):
    """The reference's own message (node/node.py:112,133: a pickled envelope
    whose 'model' is the serialized update) received into a pinned buffer:
    open_envelope hands 'model' out as a window of that buffer and land()
    reads it in place; digest = SHA-256 of the serialized update (what the
    echo signs, utils/broadcast.py:14)."""
    import hashlib

    template = {name: torch.zeros(s, device=cuda) for name, s in MLP_SHAPES}
    inbox = DeviceInbox(template, k_max=2, device=cuda)
    ser = pickle.dumps(mlp_update(11))
    env = pickle.dumps({"type": "model_update", "model": ser, "addr": "127.0.0.1", "port": 5001})
    a, b = socket.socketpair()
    th = threading.Thread(target=lambda: (a.sendall(len(env).to_bytes(4, "big") + env), a.close()))
    th.start()
    msg = inbox.recv(b)
    th.join(10)
    b.close()
    command = inbox.open_envelope(msg)
    assert command["type"] == "model_update" and command["addr"] == "127.0.0.1" and command["port"] == 5001
    assert bytes(command["model"].view()) == ser
    got = inbox.land(command["model"], digest=True)
    torch.cuda.synchronize()
    ref = pickle.loads(ser)
    for key in ref:
        assert_bits_equal(got[key].cpu().numpy(), ref[key].numpy(), what=key)
    assert inbox.digest(got.row) == hashlib.sha256(ser).digest()
    # the window keeps the buffer out of the pool until it is released
    root = command["model"].root
    assert root not in inbox._pinned_free and bytes(command["model"]) == ser
    command["model"].release()
    assert root in inbox._pinned_free
    # any other envelope decodes as the reference decodes it (pickle.loads at
    # node/node.py:112), and the buffer returns to the pool at once
    other = pickle.dumps({"type": "x", "f": collections.OrderedDict(a=1)})
    m = inbox.message_buffer(len(other))
    m.buf[:len(other)].copy_(torch.frombuffer(bytearray(other), dtype=torch.uint8))
    assert inbox.open_envelope(m) == pickle.loads(other)
    assert m.root in inbox._pinned_free


@pytest.mark.gpu
def test_pinned_landing_concurrent_listeners(cuda):
    """One listener thread per connection (node/node.py:89), each receiving
    into its own pinned buffer from the pool and landing concurrently: every
    update in its own row, bit-exact, buffers back in the pool."""
    k = 8
    template = {name: torch.zeros(s, device=cuda) for name, s in MLP_SHAPES}
    inbox = DeviceInbox(template, k_max=k, device=cuda)
    ser = [pickle.dumps(mlp_update(60 + j)) for j in range(k)]
    got = [None] * k
    barrier = threading.Barrier(k)

    def worker(j):
        barrier.wait()
        for _ in range(3):  # reuse pooled buffers while others land
            with _pinned(inbox, ser[j]) as m:  # released as the listener's frame ends
                got[j] = inbox.land(m, j)

    ths = [threading.Thread(target=worker, args=(j,)) for j in range(k)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(60)
    torch.cuda.synchronize()
    assert len({got[j].row for j in range(k)}) == k
    for j in range(k):
        ref = pickle.loads(ser[j])
        for key in ref:
            assert_bits_equal(got[j][key].cpu().numpy(), ref[key].numpy(), what=f"update {j} {key}")
    assert len(inbox._pinned_free) <= k


def test_dense_views_and_buffer_addresses():
    """Host helpers of the pinned landing path: which fp32 views can land as
    one byte run, and the address of a payload slice (writable or not)."""
    from p2pdl_amd.node.inbox import RawStorage, RawTensor, _address, _dense

    st = RawStorage(np.float32, 24, memoryview(bytearray(96)), "cpu")
    assert _dense(RawTensor(st, 0, (4, 6), (6, 1)))
    assert _dense(RawTensor(st, 3, (1, 6), (99, 1)))   # a size-1 dim may carry any stride
    assert _dense(RawTensor(st, 0, (), ()))
    assert not _dense(RawTensor(st, 0, (6, 4), (1, 6)))  # transposed
    assert not _dense(RawTensor(st, 0, (3,), (2,)))       # strided
    a = np.zeros(64, np.uint8)
    assert _address(memoryview(a)[5:9]) == a.ctypes.data + 5
    b = bytes(64)
    assert _address(memoryview(b)[7:9]) == np.frombuffer(b, np.uint8).ctypes.data + 7
