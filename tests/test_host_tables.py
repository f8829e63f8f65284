"""CPU checks of the drop-in's C gather of the peer table
(p2pdl_amd/csrc/host_tables.cpp): the lookups raise what the reference's
``received_models[j]["model"][key]`` raises (aggregator/aggregation.py:25-28),
anything the C path cannot vouch for returns 1 (the Python path diagnoses it),
and mismatched sizes are rejected before any list element is read."""
import numpy as np
import pytest
import torch

_host_tables = pytest.importorskip("p2pdl_amd._host_tables")


def _table(L, K):
    return np.zeros((L, K), dtype=np.uint64)


def test_missing_key_raises_keyerror():
    received = [{"model": {"a": torch.zeros(2)}}]
    with pytest.raises(KeyError):
        _host_tables.gather_peer_table(received, ["b", "a"], [2, 2], 0, _table(2, 1))


def test_record_without_model_raises_keyerror():
    with pytest.raises(KeyError):
        _host_tables.gather_peer_table([{"sender": 1}], ["a"], [2], 0, _table(1, 1))


def test_host_tensors_defer_to_python_path():
    received = [{"model": {"a": torch.zeros(2)}}, {"model": {"a": torch.zeros(2)}}]
    assert _host_tables.gather_peer_table(received, ["a"], [2], 0, _table(1, 2)) == 1


def test_non_tensor_defers_to_python_path():
    assert _host_tables.gather_peer_table([{"model": {"a": [0.0, 1.0]}}], ["a"], [2], 0, _table(1, 1)) == 1


@pytest.mark.parametrize("numels, shape", [([2], (2, 1)), ([2, 2], (1, 1))])
def test_size_mismatch_rejected(numels, shape):
    received = [{"model": {"a": torch.zeros(2), "b": torch.zeros(2)}}]
    with pytest.raises(ValueError):
        _host_tables.gather_peer_table(received, ["a", "b"], numels, 0, np.zeros(shape, dtype=np.uint64))


def test_sparse_tensor_defers_to_python_path():
    """the layout is checked before is_contiguous (which throws
    c10::Error on a sparse tensor and used to end in std::terminate)."""
    sp = torch.sparse_coo_tensor(torch.tensor([[0, 1]]), torch.tensor([1.0, 2.0]), (2,))
    assert _host_tables.gather_peer_table([{"model": {"a": sp}}], ["a"], [2], -1, _table(1, 1)) == 1


@pytest.mark.gpu
def test_sparse_cuda_tensor_defers_to_python_path(cuda):
    sp = torch.sparse_coo_tensor(torch.tensor([[0, 1]]), torch.tensor([1.0, 2.0]), (2,)).to(cuda)
    dense = torch.zeros(2, device=cuda)
    got = _host_tables.gather_peer_table([{"model": {"a": dense}}, {"model": {"a": sp}}], ["a"], [2],
                                         cuda.index, _table(1, 2))
    assert got == 1


def test_fill_chunk_list():
    """The split kernel's chunk list (include/p2pdl.h
    p2p_fedavg_split_chunks_f32): (segment, first element) per 1024-element
    chunk in key order, keys with no chunks skipped, the rest (-1, 0);
    -1 (nothing claimed) when the chunks do not fit."""
    nch = np.array([3, 0, 1, 2], dtype=np.int64)
    out = np.full((8, 2), 7, dtype=np.int64)
    assert _host_tables.fill_chunk_list(nch, out) == 6
    assert out.tolist() == [[0, 0], [0, 1024], [0, 2048], [2, 0], [3, 0], [3, 1024], [-1, 0], [-1, 0]]
    assert _host_tables.fill_chunk_list(np.array([9], dtype=np.int64), np.zeros((8, 2), dtype=np.int64)) == -1
    assert _host_tables.fill_chunk_list(np.array([-1], dtype=np.int64), np.zeros((8, 2), dtype=np.int64)) == -1
