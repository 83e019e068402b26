"""bench.py's code paths that only run on a GPU, checked statically on the CPU: every name a function reads is
defined in that function, an enclosing one, the module or the builtins (an undefined name in a rarely taken path,
e.g. the per-evaluation loop of --batch 1, would otherwise surface only on the GPU box)."""
import builtins
import os
import symtable

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _undefined(table, enclosing, module_names):
    bad = []
    here = {s.get_name() for s in table.get_symbols() if s.is_assigned() or s.is_parameter() or s.is_imported()
            or s.is_namespace()}
    visible = enclosing | here
    for s in table.get_symbols():
        name = s.get_name()
        if not s.is_referenced() or name in visible or name in module_names or hasattr(builtins, name):
            continue
        bad.append((table.get_name(), table.get_lineno(), name))
    for child in table.get_children():
        bad += _undefined(child, visible if table.get_type() == "function" else enclosing, module_names)
    return bad


def test_bench_has_no_undefined_names():
    path = os.path.join(ROOT, "bench.py")
    top = symtable.symtable(open(path).read(), path, "exec")
    module_names = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()
                    or s.is_namespace()}
    bad = []
    for child in top.get_children():
        bad += _undefined(child, set(), module_names)
    assert not bad, f"undefined names in bench.py (function, line, name): {bad}"
