"""Every global name a function of the GPU-only scripts reads is defined.

bench.py's records and most of p2pdl_amd run only on the GPU box; a name
error in one of them surfaces there, late.  symtable gives each scope's free
and implicit-global references; each must be a module-level binding or a
builtin."""
import builtins
import pathlib
import symtable

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
FILES = ["bench.py", "__graft_entry__.py"] + sorted(str(p.relative_to(ROOT)) for p in (ROOT / "p2pdl_amd").rglob("*.py"))


def _undefined(path):
    src = (ROOT / path).read_text()
    top = symtable.symtable(src, path, "exec")
    defined = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()
               or s.is_namespace()}
    known = defined | set(dir(builtins)) | {"__file__", "__name__", "__doc__", "__spec__", "__builtins__"}
    bad = []

    def walk(t):
        for s in t.get_symbols():
            if t.get_type() != "module" and s.is_referenced() and s.is_global() and not s.is_declared_global() \
                    and s.get_name() not in known:
                bad.append(f"{t.get_name()}:{s.get_name()}")
        for c in t.get_children():
            walk(c)

    walk(top)
    return bad


@pytest.mark.parametrize("path", FILES)
def test_no_undefined_globals(path):
    assert _undefined(path) == []
