"""CPU: the C-ABI library loads (no GPU needed) and exports every symbol include/recsys_amd.h
declares, with the argument counts the ctypes binding uses."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "recsys_amd.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(?:int|int64_t)\s+(rs_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        args = [a.strip() for a in m.group(2).split(",") if a.strip() not in ("", "void")]
        out[m.group(1)] = len(args)
    return out


def test_header_parses():
    d = declared()
    assert len(d) >= 15 and "rs_il_fwd" in d and "rs_embedding_lookup_fwd" in d


def test_library_exports_every_declared_symbol():
    from recommendsystem_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = _lib.load()
    for name in declared():
        assert hasattr(lib, name), f"{name} not exported"


def test_binding_matches_header():
    from recommendsystem_amd._lib import SIGNATURES
    d = declared()
    assert set(d) == set(SIGNATURES), set(d) ^ set(SIGNATURES)
    for name, n in d.items():
        assert len(SIGNATURES[name][1]) == n, name


def test_host_only_entry_points():
    """Pure host-side entry points are callable without a GPU."""
    from recommendsystem_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    lib = _lib.load()
    assert lib.rs_il_param_count(16, 16) == 16 * 64 + 64 + 32
    assert lib.rs_il_bwd_workspace_floats(4096, 16, 16) >= 1120
    assert lib.rs_dense_bwd_weight_workspace_floats(4096, 416, 32) % (416 * 32 + 32) == 0


def test_missing_library_fails_loudly(tmp_path):
    from recommendsystem_amd import _lib
    with pytest.raises(_lib.RecsysKernelError):
        _lib.load.__wrapped__(str(tmp_path / "nope.so")) if hasattr(_lib.load, "__wrapped__") else \
            _load_fresh(str(tmp_path / "nope.so"))


def _load_fresh(path):
    from recommendsystem_amd import _lib
    saved = _lib._LIB
    _lib._LIB = None
    try:
        _lib.load(path)
    finally:
        _lib._LIB = saved
