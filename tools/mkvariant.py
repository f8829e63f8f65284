#!/usr/bin/env python3
"""Build an A/B variant of the product library without touching product source.

usage: python tools/mkvariant.py <name> <patch.py>
Copies p2pdl_amd/csrc + include into /tmp/p2p_variant_<name>, runs the patch
script there (it edits files relative to the copy's csrc directory, and must
assert that each replacement matched), builds the library and installs it as
tools/libp2pdl_<name>.so.  Select it with P2P_LIB=tools/libp2pdl_<name>.so
(tools/gpu_ab_sq.sh, bench.py).
"""
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    name, patch = sys.argv[1], os.path.abspath(sys.argv[2])
    root = f"/tmp/p2p_variant_{name}"
    shutil.rmtree(root, ignore_errors=True)
    shutil.copytree(os.path.join(REPO, "include"), os.path.join(root, "include"))
    shutil.copytree(os.path.join(REPO, "p2pdl_amd", "csrc"), os.path.join(root, "p2pdl_amd", "csrc"),
                    ignore=shutil.ignore_patterns("build"))
    csrc = os.path.join(root, "p2pdl_amd", "csrc")
    subprocess.run([sys.executable, patch], cwd=csrc, check=True)
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-j", jobs, "../libp2pdl_hip.so"], cwd=csrc, check=True, stdout=subprocess.DEVNULL)
    out = os.path.join(REPO, "tools", f"libp2pdl_{name}.so")
    shutil.copy(os.path.join(root, "p2pdl_amd", "libp2pdl_hip.so"), out)
    print(out)


if __name__ == "__main__":
    main()
