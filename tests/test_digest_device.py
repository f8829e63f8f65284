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
