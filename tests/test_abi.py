"""The C-ABI library loads and exports every symbol include/afm.h declares (no GPU needed)."""
import ctypes
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "afm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(afm_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from afm import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    names = header_functions()
    assert len(names) >= 7
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)


def test_factor_names_match_reference_order():
    import oracle
    from afm import FACTOR_NAMES, _lib
    assert _lib.factor_names() == FACTOR_NAMES == oracle.FACTOR_NAMES
    g = np.load(os.path.join(ROOT, "tests", "golden", "factors_edge.npz"))
    assert list(g["all_cols"]) == FACTOR_NAMES


def test_errors_do_not_throw_without_gpu():
    from afm import _lib
    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.afm_ctx_create(123456, ctypes.byref(h))
    assert rc != 0 and len(L.afm_last_error()) > 0
    assert L.afm_ctx_destroy(None) != 0
    assert L.afm_version() >= 1


def test_bit_packing_roundtrip():
    import torch
    from afm import pack_bits, unpack_bits
    from afm.synthetic import unpack_bits as np_unpack, valid_bits
    rng = np.random.default_rng(0)
    v = rng.random((197, 128)) < 0.7
    b = pack_bits(torch.from_numpy(v))
    assert np.array_equal(unpack_bits(b, 197).numpy(), v)
    assert np.array_equal(b.numpy().view(np.uint64), valid_bits(v))
    assert np.array_equal(np_unpack(valid_bits(v), 197), v)
