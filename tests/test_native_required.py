"""No silent host fallbacks: the product imports its host
extensions -- ``_host_tables`` (the drop-in's peer-table gather,
csrc/host_tables.cpp) and ``_wire`` (the receive path's restricted pickle
machine, csrc/wire.cpp) -- unconditionally.  A build that did not produce one
fails at import with NativeUnavailable instead of running the slower Python
paths; the Python machine stays only as the tests' differential reference."""
import subprocess
import sys

import pytest

ROOT = __import__("pathlib").Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("ext,module", [("_wire", "p2pdl_amd.node.inbox"),
                                        ("_host_tables", "p2pdl_amd.aggregator.aggregation")])
def test_import_without_host_extension_fails_loudly(ext, module):
    code = f"""
import sys
sys.modules["p2pdl_amd.{ext}"] = None  # as if the .so were missing: import raises ImportError
from p2pdl_amd._native import NativeUnavailable
try:
    import {module}
except NativeUnavailable as e:
    assert "{ext}" in str(e) and "make -C p2pdl_amd/csrc" in str(e), e
    print("LOUD")
else:
    print("SILENT")
"""
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().endswith("LOUD"), r.stdout + r.stderr


def test_extensions_are_the_built_ones():
    """With the build in place both import from the package directory."""
    from p2pdl_amd import _host_tables, _wire
    from p2pdl_amd.node import inbox

    assert inbox._wire is _wire
    assert _wire.__file__.startswith(str(ROOT / "p2pdl_amd"))
    assert _host_tables.__file__.startswith(str(ROOT / "p2pdl_amd"))
    assert inbox.ZeroCopyParser(b"").native is True
