"""utils.digests.digest_device_messages: SHA-256 of messages resident in
device memory by the measured boundary -- the GPU batch kernel for many
short messages, the host threads with pipelined D2H for long ones --
byte-equal to hashlib on both routes (unaligned offsets, empty messages,
lengths around the staging piece size)."""
import hashlib

import numpy as np
import pytest
import torch

from p2pdl_amd.utils import digests as dg


def _buffer(lengths, seed, cuda):
    rng = np.random.default_rng(seed)
    offs, o = [], 3  # odd start: unaligned messages
    for n in lengths:
        offs.append(o)
        o += n + 5
    host = rng.integers(0, 256, size=o + 8, dtype=np.uint8)
    return torch.from_numpy(host).to(cuda), host, offs


@pytest.mark.gpu
@pytest.mark.parametrize("lengths", [
    [0, 1, 55, 56, 64, 1000],                                     # few messages: host route
    [dg.STAGE - 1, dg.STAGE, dg.STAGE + 1, 2 * dg.STAGE + 77],    # staging piece boundaries
    [100 + (i * 37) % 9000 for i in range(dg.GPU_BATCH_MIN)],     # many short ones: the GPU kernel
])
def test_device_message_digests_match_hashlib(cuda, lengths):
    dev, host, offs = _buffer(lengths, len(lengths), cuda)
    got = dg.digest_device_messages(dev, offs, lengths).cpu().numpy()
    for i, (o, n) in enumerate(zip(offs, lengths)):
        assert bytes(got[i]) == hashlib.sha256(host[o:o + n].tobytes()).digest(), (i, n)


@pytest.mark.gpu
def test_device_message_digests_see_the_callers_stream(cuda):
    """The host route waits for work the caller queued on its stream."""
    n = 3 * dg.STAGE
    dev = torch.zeros(n, dtype=torch.uint8, device=cuda)
    s = torch.cuda.Stream(cuda)
    with torch.cuda.stream(s):
        torch.cuda._sleep(50_000_000)
        dev.fill_(7)
        got = dg.digest_device_messages(dev, [0], [n]).cpu().numpy()
    assert bytes(got[0]) == hashlib.sha256(bytes([7]) * n).digest()


@pytest.mark.parametrize("offsets,lengths,why", [
    ([0, 90], [10, 11], "outside"),     # ends one byte past the buffer
    ([-1], [4], "outside"),             # negative offset
    ([0], [-1], "outside"),             # negative length
    ([0, 1], [1], "offsets for"),       # count mismatch
])
def test_message_spans_are_checked_before_any_device_read(offsets, lengths, why):
    """The kernel reads raw addresses: a span outside the buffer is a
    ValueError on the host, never a launch (no GPU needed to check)."""
    from p2pdl_amd import ops

    buf = torch.zeros(100, dtype=torch.uint8)
    with pytest.raises(ValueError, match=why):
        ops.check_message_spans(buf, offsets, lengths)
    ops.check_message_spans(buf, [0, 90, 100], [90, 10, 0])  # the edges themselves are inside


@pytest.mark.parametrize("bad", [torch.zeros(8, dtype=torch.float32), torch.zeros((2, 8), dtype=torch.uint8),
                                 torch.zeros(16, dtype=torch.uint8)[::2]])
def test_message_buffer_must_be_flat_bytes(bad):
    from p2pdl_amd import ops

    with pytest.raises(ValueError, match="contiguous 1-D uint8"):
        ops.check_message_spans(bad, [0], [1])


def test_fused_path_wrappers_check_shapes_before_the_launch():
    """digest_accept / fedavg_apply_devk_ pass raw addresses to kernels that
    index k rows: a mis-sized operand is a ValueError on the host (checked
    here with host tensors; the checks run before any native call)."""
    from p2pdl_amd import ops

    k = 4
    dig, exp = torch.zeros((k, 32), dtype=torch.uint8), torch.zeros((k, 32), dtype=torch.uint8)
    tbl, acc, cnt = torch.zeros(k, dtype=torch.int64), torch.zeros(k, dtype=torch.int64), torch.zeros(1, dtype=torch.int32)
    for args, what in [((dig[:3], exp, tbl, acc, cnt), "digests"), ((dig, exp[:, :16], tbl, acc, cnt), "expected"),
                       ((dig, exp, tbl, acc[:3], cnt), "accepted"), ((dig, exp, tbl, acc, cnt[:0]), "count"),
                       ((dig, exp, tbl.int(), acc, cnt), "payload_table")]:
        with pytest.raises(ValueError, match=what):
            ops.digest_accept(*args)
    w = torch.zeros(10)
    with pytest.raises(ValueError, match="table"):
        ops.fedavg_apply_devk_(w, tbl[:2], cnt, 3)
    with pytest.raises(ValueError, match="k_dev"):
        ops.fedavg_apply_devk_(w, tbl, cnt.long(), 3)
    with pytest.raises(ValueError, match="out has"):
        ops.fedavg_apply_devk_(w, tbl, cnt, 3, out=torch.zeros(9))


@pytest.mark.gpu
def test_cfg5_product_route_at_k256(cuda):
    """cfg5 at its configuration's K (VERDICT r04 next #3a): 256 device-
    resident serialized updates of >= 2 staging pieces each, ~10% corrupted,
    through the product route bench.py's cfg5 times --
    digest_device_messages (host SHA threads, pipelined D2H) -> digest_accept
    -> fedavg_apply_devk_ (K from the device, k_max = 256) -- against
    hashlib (what the senders signed, node/node.py:285 -> utils/crypto.py:56)
    and the FedAvg oracle over the accepted updates in list order
    (aggregation.py:15-38)."""
    import oracle  # checker only
    from p2pdl_amd import ops

    K, hdr = 256, 64
    n = (2 * dg.STAGE + 12345) // 4  # fp32 payload: each message spans 3 staging pieces
    msg = hdr + 4 * n
    stride = -(-msg // 256) * 256
    seed = 0x5EED0C05
    buf = torch.zeros(K * stride, dtype=torch.uint8, device=cuda)
    offsets = [p * stride for p in range(K)]
    for p in range(K):
        buf[offsets[p]:offsets[p] + hdr] = torch.tensor(list((b"update %05d " % p).ljust(hdr, b"\0")),
                                                       dtype=torch.uint8, device=cuda)
        ops.fill_synthetic_(buf[offsets[p] + hdr:offsets[p] + msg].view(torch.float32), seed, p, 1e-2)
    host = buf.cpu().numpy()
    signed = [hashlib.sha256(host[o:o + msg].tobytes()).digest() for o in offsets]
    expected = torch.tensor(np.frombuffer(b"".join(signed), dtype=np.uint8).reshape(K, 32), device=cuda)
    bad = [p for p in range(K) if (p * 7919) % 10 == 3]
    for p in bad:  # corrupted in flight: one payload byte
        buf[offsets[p] + hdr + 1000 + p] ^= 0x40
    digests = dg.digest_device_messages(buf, offsets, [msg] * K)
    got = digests.cpu().numpy()
    for p in range(K):
        assert (bytes(got[p]) == signed[p]) == (p not in bad), p
    payload_tbl = torch.tensor([buf.data_ptr() + o + hdr for o in offsets], dtype=torch.int64, device=cuda)
    accepted = torch.zeros(K, dtype=torch.int64, device=cuda)
    count = torch.zeros(1, dtype=torch.int32, device=cuda)
    w = torch.empty(n, dtype=torch.float32, device=cuda)
    ops.fill_synthetic_(w, seed, 0xFFFFF, 5e-2)
    ops.digest_accept(digests, expected, payload_tbl, accepted, count)
    ops.fedavg_apply_devk_(w, accepted, count, K)
    keep = [p for p in range(K) if p not in bad]
    assert int(count.item()) == len(keep)
    tbl = payload_tbl.cpu().tolist()
    assert accepted.cpu().tolist()[:len(keep)] == [tbl[p] for p in keep]  # list order
    wh = w.cpu().numpy()
    for a, b in [(0, 5000), (n // 2, n // 2 + 9000), (n - 70_000, n)]:
        idx = np.arange(a, b)
        want, _ = oracle.fedavg([oracle.synth_at(idx, seed, p, 1e-2) for p in keep],
                                oracle.synth_at(idx, seed, 0xFFFFF, 5e-2))
        assert np.array_equal(wh[a:b].view(np.uint32), want.view(np.uint32)), (a, b)
