"""Static check over the package and the entry scripts: every name a function reads must be bound
somewhere -- a local, an enclosing function's, a module global or a builtin (symtable, no
imports executed).  Catches a renamed local left behind in a code path no CPU test runs (the GPU
backward of the ResNet stem read a name an edit had renamed)."""
import builtins
import pathlib
import symtable

ROOT = pathlib.Path(__file__).resolve().parent.parent
FILES = sorted(p for p in (ROOT / "kungfu_amd").rglob("*.py")) + [ROOT / "bench.py", ROOT / "__graft_entry__.py"]


def _module_names(top):
    names = set(top.get_identifiers())
    return names


def _walk(tab, module_names, path, bad):
    for child in tab.get_children():
        if child.get_type() == "function":
            for sym in child.get_symbols():
                if not sym.is_referenced():
                    continue
                if sym.is_global() and not sym.is_declared_global():
                    n = sym.get_name()
                    if n not in module_names and not hasattr(builtins, n) and n not in ("__class__",):
                        bad.append("%s: %s() reads unbound name %r" % (path.relative_to(ROOT), child.get_name(), n))
        _walk(child, module_names, path, bad)


def test_no_unbound_names():
    bad = []
    for p in FILES:
        src = p.read_text()
        top = symtable.symtable(src, str(p), "exec")
        _walk(top, _module_names(top), p, bad)
    assert not bad, "\n".join(bad)
