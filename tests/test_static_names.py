"""Undefined-name check of the Python host code that only a GPU box runs end
to end (bench.py's multi-rank step and self-checks, the ShardedQuery
exchanges): every implicitly global name a function reads must be a module
global or a builtin.  A NameError there (a helper module not in scope) would
otherwise surface only in the driver's GPU bench.  CPU only, stdlib symtable.
"""
from __future__ import annotations

import builtins
import os
import symtable

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = ["bench.py", "__graft_entry__.py", "warpdb_amd/distributed.py", "warpdb_amd/_warpexec.py"]


def _undefined(path: str):
    src = open(path).read()
    top = symtable.symtable(src, path, "exec")
    module_names = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported() or s.is_global()}
    module_names |= {c.get_name() for c in top.get_children()}
    bad = []

    def walk(t):
        for s in t.get_symbols():
            if t.get_type() == "function" and s.is_global() and not s.is_declared_global():
                n = s.get_name()
                if n not in module_names and not hasattr(builtins, n) and n != "__file__":
                    bad.append((t.get_name(), t.get_lineno(), n))
        for c in t.get_children():
            walk(c)

    walk(top)
    return bad


@pytest.mark.parametrize("rel", FILES)
def test_no_undefined_names(rel):
    assert _undefined(os.path.join(ROOT, rel)) == []
