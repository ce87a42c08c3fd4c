"""CPU: the C-ABI library loads and exports every symbol include/*.h declares.

No compute call is made here (there is no GPU in the build container); the device paths
are covered by tests/test_gpu_parity.py (marked gpu).
"""
import ctypes as C
import os
import re

import pytest

from titan_amd import _lib as L

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def declared_functions():
    names = set()
    for h in os.listdir(os.path.join(ROOT, "include")):
        if not h.endswith(".h"):
            continue
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(tgo_[a-z_0-9]+)\s*\(", src):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    lib = L.load()
    decl = declared_functions()
    assert decl, "no declarations found"
    missing = [n for n in sorted(decl) if not hasattr(lib, n)]
    assert not missing, missing
    assert decl == set(L.EXPORTS)


def test_struct_layouts_match_header():
    # sizes of the by-value structs as the C compiler lays them out
    assert C.sizeof(L.Options) == 32
    assert C.sizeof(L.Rows) == 48
    assert C.sizeof(L.LoadOpts) == 32
    assert C.sizeof(L.BfsArgs) == 24
    assert C.sizeof(L.SsspArgs) == 40
    assert C.sizeof(L.PrArgs) == 24
    assert C.sizeof(L.EdgeEntry) == 32
    # tgo_edge_type: sort_order fills the slot after n_signature (no size change)
    assert C.sizeof(L.EdgeType) == 40
    assert L.EdgeType.sort_order.offset == 28 and L.EdgeType.signature_ids.offset == 32


def test_default_options():
    lib = L.load()
    o = L.Options()
    lib.tgo_default_options(C.byref(o))
    assert o.abi_version == L.ABI_VERSION
    assert o.partition_bits == 5 and o.hard_query_limit == 100000


def test_create_fails_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    lib = L.load()
    o = L.Options()
    lib.tgo_default_options(C.byref(o))
    h = C.c_void_p()
    assert lib.tgo_create(C.byref(o), C.byref(h)) == L.TGO_E_HIP
    assert not h.value


def test_last_error_on_null_ctx():
    lib = L.load()
    assert lib.tgo_last_error(None) == b"null ctx"


def test_rmat_generator_is_deterministic_and_in_range():
    from titan_amd import rmat_edges
    s1, d1, w1 = rmat_edges(10, 16, seed=5, weights=True, threads=3)
    s2, d2, w2 = rmat_edges(10, 16, seed=5, weights=True, threads=1)
    assert (s1 == s2).all() and (d1 == d2).all() and (w1 == w2).all()
    assert s1.min() >= 0 and s1.max() < 1024 and d1.max() < 1024
    assert w1.min() >= 1 and w1.max() <= 255
    # RMAT skew: the top vertex holds far more than the average degree
    import numpy as np
    deg = np.bincount(np.concatenate([s1, d1]), minlength=1024)
    assert deg.max() > 8 * deg.mean()
