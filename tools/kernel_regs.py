#!/usr/bin/env python3
"""Register / scratch / LDS use per kernel of a hipcc-built shared library.

usage: python tools/kernel_regs.py <lib.so> [name-substring ...]

Reads the AMDGPU metadata notes of every gfx950 code object in the library's
offload bundles (llvm-readobj --notes): .vgpr_count, .agpr_count,
.sgpr_count, .private_segment_fixed_size (scratch bytes per lane) and
.group_segment_fixed_size (static LDS bytes).
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_stats  # noqa: E402

LLVM = isa_stats.LLVM
KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".private_segment_fixed_size", ".group_segment_fixed_size")


def kernels(path):
    fat = isa_stats.fatbin_of_so(path)
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [i for i in range(0, len(fat), 4096) if fat.startswith(magic, i)]
    out = {}
    for a, b in zip(starts, starts[1:] + [len(fat)]):
        with tempfile.TemporaryDirectory() as d:
            bundle, co = os.path.join(d, "b"), os.path.join(d, "co")
            with open(bundle, "wb") as f:
                f.write(fat[a:b])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={bundle}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
            notes = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
        cur = {}
        for line in notes.splitlines():
            s = line.strip().lstrip("- ")
            m = re.match(r"(\.[a-z_]+):\s+(\S+)", s)
            if not m:
                continue
            k, v = m.groups()
            if k in KEYS:
                cur[k] = v
            elif k == ".name" and not v.endswith(".kd"):
                cur = {}
                out[v] = cur
    return out


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    for name, d in sorted(kernels(path).items()):
        if subs and not any(s in name for s in subs):
            continue
        print(f"{name}: vgpr={d.get('.vgpr_count')} agpr={d.get('.agpr_count')} sgpr={d.get('.sgpr_count')} "
              f"scratch={d.get('.private_segment_fixed_size')} lds={d.get('.group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
