"""The C-ABI library loads on a GPU-less host and exports every declared symbol."""
import os
import re
import subprocess

from p2pdl_amd import _native as N

HEADER = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "p2pdl.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(p2p_\w+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_functions() == sorted(N.EXPORTS)


def test_library_exports_every_declared_symbol():
    N.load_library()
    out = subprocess.check_output(["nm", "-D", "--defined-only", N.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    internal = [s for s in exported if s.startswith("p2p_") and s not in declared_functions()]
    assert not internal, f"undeclared exports: {internal}"


def test_abi_version_and_argument_errors_without_gpu():
    L = N.load_library()
    assert L.p2p_abi_version() == N.ABI_VERSION
    assert L.p2p_strerror(0) == b"ok"
    assert b"invalid" in L.p2p_strerror(-1)
    # tile sizes are a pure function of (rule, k): no process-wide layout state
    assert L.p2p_tile_elems(0, 3) == 4096 and L.p2p_tile_elems(0, 256) == 4096
    assert L.p2p_tile_elems(1, 64) == 128 and L.p2p_tile_elems(1, 128) == 128
    # K > 128: the median pair kernel runs two wave pairs (128 coordinates)
    # per block; the trimmed mean's pair and LDS kernels share 64
    assert L.p2p_tile_elems(1, 129) == 128 and L.p2p_tile_elems(1, 256) == 128
    assert L.p2p_tile_elems(2, 200) == 64 and L.p2p_tile_elems(2, 256) == 64
    assert L.p2p_tile_elems(3, 3) == 4096 and L.p2p_tile_elems(3, 300) == 4096  # FedAvg, torch-GPU division
    assert L.p2p_aggregate_f32(1, 3, 0, 4, 0, 0.1, 16, None, None) == -1  # no rule 4
    assert L.p2p_aggregate_segments_f32(1, 1, 0, 3, 4, 0, 0.1, None) == -1
    # argument validation happens before any HIP call
    assert L.p2p_fedavg_apply_f32(None, 3, 10, None, 0.1, None) == N.lib().p2p_aggregate_f32(
        None, 1, 1, 0, 0, 0.1, None, None, None) == -1
    assert L.p2p_median_f32(1, 300, 10, 16, None) == -2  # k > 256 unsupported
    assert L.p2p_trimmed_mean_f32(1, 4, 10, 2, 16, None) == -1  # K - 2b == 0
    assert L.p2p_apply_f32(2, 16, 0.1, 10, None) == -3  # misaligned w
    # ABI 9: launch hints; unknown bits are refused before any HIP call
    assert L.p2p_aggregate_ex_f32(1, 3, 0, 0, 0, 0.1, 16, None, 2, None) == -1
    assert L.p2p_aggregate_ex_f32(1, 3, 0, 0, 0, 0.1, 16, None, N.P2P_HINT_SHARE_CUS, None) == 0  # n = 0: nothing
    assert L.p2p_fedavg_split_chunks_f32(None, 1, 16, 16, 0, 0.1, None) == -1
    assert L.p2p_fedavg_split_chunks_f32(16, 1, 16, 16, 1, 0.1, None) == -1  # robust rule: not on the split kernel
