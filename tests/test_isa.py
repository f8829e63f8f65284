"""ISA checks of the built library: the robust kernels' NaN handling does not
rest on what -fno-honor-nans lets the compiler assume.

The robust objects are built with -mno-amdgpu-ieee -fno-honor-nans so the
float network's v_min/v_max need no canonicalisation (robust_nets.h).  NaN is
still a specified input class: a wave (or pair block) holding one must take
the uint32-key network.  These checks read the code object inside
p2pdl_amd/libp2pdl_hip.so (llvm-objdump, tools/isa_stats.py) and assert
  * every function that runs the float network also issues the explicit NaN
    test over every key it loads (asm v_pk_fma_f32 chains, through which NaN
    propagates, ended by a v_cmp_u_f32; or one compare per two keys) -- the
    compiler would fold an isnan() away under this flag, asm it cannot; the
    pair kernels instead compare their sorts' rank-0 outputs, whose cones are
    asm v_minimum3_f32 throughout (gen_networks.py asserts the cone holds
    only mins and reaches every input);
  * every key-path function (pair_keys, robust_coord_keys) and every MODE 0
    kernel sorts with integer min / max / med3 only, so a NaN key is ranked
    by its bits whatever the float mode;
  * the float path never holds a NaN: no float min / max in a function
    without the NaN test.
No GPU needed; the parity of both paths is the GPU suite's job.
"""
import collections
import os
import re
import shutil
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import isa_stats  # noqa: E402

SO = os.path.join(REPO, "p2pdl_amd", "libp2pdl_hip.so")
FLOAT_MINMAX = ("v_min_f32", "v_max_f32", "v_med3_f32", "v_min3_f32", "v_max3_f32")
INT_MINMAX = ("v_min_u32", "v_max_u32", "v_med3_u32", "v_min3_u32", "v_max3_u32")


@pytest.fixture(scope="module")
def funcs():
    if not os.path.exists(SO):
        pytest.fail(f"{SO} is not built (python -c 'import __graft_entry__ as g; g.build()')")
    if not os.path.exists(os.path.join(isa_stats.LLVM, "llvm-objdump")) or shutil.which("true") is None:
        pytest.skip("ROCm LLVM tools not installed")
    out = {}
    for name, ops in isa_stats.functions(isa_stats.disassemble(SO)).items():
        out[name] = collections.Counter(ops)
    return out


def _count(c, names):
    return sum(c[n] for n in names) + sum(v for k, v in c.items() if k.startswith(tuple(n + "_e" for n in names)))


def _mode(name):
    """MODE template argument of robust_flat / robust_segments kernels (0 = generic key network)."""
    m = re.search(r"robust_(?:flat|segments)_kernelILi(\d+)ELi(\d)ELi(\d)E", name)
    return (int(m.group(1)), int(m.group(3))) if m else None


def test_robust_kernels_present(funcs):
    names = " ".join(funcs)
    for k in ("robust_median_pair_kernel", "robust_pair_kernel", "robust_flat_kernel", "robust_segments_kernel",
              "robust_lds_g2_kernel", "pair_keys", "robust_coord_keys"):
        assert k in names, k


def test_float_network_always_behind_the_nan_test(funcs):
    checked = 0
    for name, c in funcs.items():
        if "robust" not in name and "pair_keys" not in name:
            continue
        if _count(c, FLOAT_MINMAX) == 0:
            continue
        cmps = c["v_cmp_u_f32"] + c["v_cmp_u_f32_e64"] + c["v_cmp_u_f32_e32"]
        pk = c["v_pk_fma_f32"]
        mx = c["v_maximum3_f32"]
        # the loads of the function: one per key (pair: 128 per wave, K <= 128: KP).
        # robust_nets.h nan_lanes: a chain of packed FMAs folds 6 keys, then 4
        # per instruction, into a pair that one compare tests; the padded
        # kernels' slots that may hold +-inf pad rows fold 2 keys per
        # v_maximum3_f32 instead; plain compares test 2 keys each -- either way
        # 4 * pk + 2 * mx + 2 * cmps keys are covered (each chain's compare
        # counts the two extra keys its first instruction folds); the loads
        # include one that is not a key (the w read of the apply)
        loads = sum(v for k, v in c.items() if k.startswith("global_load") and "lds" not in k)
        # the pair kernels' rank-0 cones: 76 NaN-propagating mins per sort128,
        # 36 per sort64 (two per median wave)
        rank0 = c["v_minimum3_f32"] >= 72
        assert cmps > 0 and (rank0 or 4 * pk + 2 * mx + 2 * cmps >= loads - 1 > 0), (name, cmps, pk, mx, loads)
        checked += 1
    assert checked >= 6


def test_key_paths_are_integer_networks(funcs):
    checked = 0
    for name, c in funcs.items():
        km = _mode(name)
        if "pair_keys" in name or "robust_coord_keys" in name or (km and km[1] == 0 and km[0] >= 8):
            assert _count(c, FLOAT_MINMAX) == 0, (name, {k: c[k] for k in FLOAT_MINMAX})
            assert _count(c, INT_MINMAX) > 0, name
            checked += 1
    assert checked >= 8


def test_no_scalar_memory_writes_anywhere(funcs):
    """No function of the library writes through the scalar data cache (no
    scalar stores, scalar atomics or scalar-cache write-back / discard): every
    store, and the tile queue's claim atomics, are vector memory ops."""
    bad = {name: [op for op in c if op.startswith(("s_store", "s_buffer_store", "s_atomic", "s_buffer_atomic",
                                                    "s_dcache_wb", "s_dcache_discard", "s_scratch_store"))]
           for name, c in funcs.items()}
    bad = {k: v for k, v in bad.items() if v}
    assert not bad, bad


def test_split_kernel_modes_and_queue_present(funcs):
    """The split kernel's modes (flat 0, segments 1, rows 2, chunks 3) are
    built with and without the tile queue; the queued ones claim tiles with a
    vector atomic add; the chunk list's loaders DMA through buffer loads
    (lanes past a key's end masked by the descriptor)."""
    split = {n: c for n, c in funcs.items() if "fedavg_split_kernel" in n}
    for mode in range(4):
        for q in (0, 1):
            assert any(f"ILb0ELi{mode}ELb{q}E" in n for n in split), (mode, q)
    for n, c in split.items():
        if "ELb1EE" in n:  # QUEUE
            assert c["global_atomic_add"] + c["global_atomic_add_u32"] + sum(
                v for k, v in c.items() if k.startswith("global_atomic_add")) >= 1, n
        if "ELi3E" in n:  # CHUNKS
            assert sum(v for k, v in c.items() if k.startswith("buffer_load_dwordx4")) >= 1, n
