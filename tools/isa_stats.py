#!/usr/bin/env python3
"""Static instruction counts per device function of a gfx950 object.

usage: python tools/isa_stats.py <hipcc -c output (bundle) or .co> [name-substring ...]

Unbundles the gfx950 code object (clang-offload-bundler), disassembles it
(llvm-objdump) and prints, per function: VALU / SALU / VMEM / LDS / scratch
instruction counts and barriers.  Static counts: a loop body counts once.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def fatbin_of_so(path: str) -> bytes:
    """The .hip_fatbin section of a hipcc-built shared library (an offload bundle)."""
    out = subprocess.run([f"{LLVM}/llvm-readelf", "-S", "--wide", path], check=True, capture_output=True,
                         text=True).stdout
    for line in out.splitlines():
        if ".hip_fatbin" in line:
            f = line.split("]", 1)[1].split()
            off, size = int(f[3], 16), int(f[4], 16)
            with open(path, "rb") as fh:
                fh.seek(off)
                return fh.read(size)
    raise ValueError(f"{path}: no .hip_fatbin section")


def disassemble(path: str) -> str:
    with open(path, "rb") as f:
        head = f.read(24)
    if head.startswith(b"\x7fELF") and path.endswith(".so"):
        # one offload bundle per translation unit, concatenated (4 KiB aligned)
        fat = fatbin_of_so(path)
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [i for i in range(0, len(fat), 4096) if fat.startswith(magic, i)]
        parts = []
        for a, b in zip(starts, starts[1:] + [len(fat)]):
            tmpso = tempfile.NamedTemporaryFile(suffix=".bundle", delete=False)
            tmpso.write(fat[a:b])
            tmpso.close()
            try:
                parts.append(disassemble(tmpso.name))
            finally:
                os.unlink(tmpso.name)
        return "\n".join(parts)
    tmp = None
    if head.startswith(b"__CLANG_OFFLOAD_BUNDLE__"):
        tmp = tempfile.NamedTemporaryFile(suffix=".co", delete=False)
        tmp.close()
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={path}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={tmp.name}"], check=True)
        path = tmp.name
    try:
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", path],
                              check=True, capture_output=True, text=True).stdout
    finally:
        if tmp:
            os.unlink(tmp.name)


def functions(asm: str):
    out = collections.OrderedDict()
    cur = None
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        s = line.strip()
        if cur and s and not s.startswith(";"):
            out[cur].append(s.split()[0])
    return out


def stats(ops):
    c = collections.Counter(ops)

    def n(pred):
        return sum(v for k, v in c.items() if pred(k))
    return {
        "total": len(ops),
        "valu": n(lambda k: k.startswith("v_") and not k.startswith("v_mfma")),
        "salu": n(lambda k: k.startswith("s_") and not k.startswith(("s_load", "s_buffer", "s_waitcnt", "s_barrier",
                                                                      "s_cbranch", "s_branch", "s_nop"))),
        "vmem": n(lambda k: k.startswith(("global_", "buffer_", "flat_"))),
        "lds": n(lambda k: k.startswith("ds_")),
        "scratch": n(lambda k: k.startswith("scratch_") or ("buffer_" in k and "lds" not in k and False)),
        "barrier": c["s_barrier"],
        "calls": c["s_swappc_b64"],
    }, c


def main():
    path, filters = sys.argv[1], sys.argv[2:]
    for name, ops in functions(disassemble(path)).items():
        if filters and not any(f in name for f in filters):
            continue
        st, _ = stats(ops)
        print(name[:100], " ".join(f"{k}={v}" for k, v in st.items()))


if __name__ == "__main__":
    main()
