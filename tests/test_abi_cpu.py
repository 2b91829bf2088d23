"""CPU-side checks of the drop-in boundary: libmtts.so loads (no GPU needed to
dlopen) and exports exactly the entry points include/*.h declare."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    out = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if not h.endswith(".h"):
            continue
        with open(os.path.join(ROOT, "include", h)) as f:
            txt = f.read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        out |= set(re.findall(r"\b(mtts_[a-z0-9_]+)\s*\(", txt))
    return sorted(out)


def test_header_and_binding_agree():
    from moss_tts_amd import _native
    assert set(declared_symbols()) == set(_native.EXPORTED)


def test_library_exports_every_declared_symbol():
    from moss_tts_amd import _native
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libmtts.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_native.lib_path())
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    _native.load()
    assert lib.mtts_version() == 1


def test_errors_map_to_reference_exceptions():
    from moss_tts_amd import _native
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libmtts.so not built")
    _native.load()
    # null config -> MTTS_E_INVALID -> ValueError (the reference raises ValueError on bad inputs)
    with pytest.raises(ValueError):
        _native.check(_native.load().mtts_engine_create(None, 0, None), "create")
    with pytest.raises(ValueError):
        _native.check(_native.load().mtts_codec_create(None, 0, None), "codec create")


def test_packed_gemm_argument_checks():
    """mtts_k_gemm_packed refuses shapes its kernels do not take, before any device call:
    K % 64 != 0, fewer than 33 rows, a packed output for a non-SwiGLU epilogue."""
    from moss_tts_amd import _native
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libmtts.so not built")
    L = _native.load()
    for M, K, epi, ypk in [(181, 96, 0, 0), (32, 4096, 0, 0), (181, 4096, 1, 1), (181, 4096, 7, 0)]:
        with pytest.raises(ValueError):
            _native.check(L.mtts_k_gemm_packed(None, None, None, 16, ypk, None, 16, M, 16, K, epi, None, 1, None, 0,
                                               None), "gemm_packed")


def test_rope_table_host_path():
    """mtts_rope_table is host code: check it against the oracle on the CPU."""
    import numpy as np
    from moss_tts_amd import _native
    from oracle import bf16 as B16
    from oracle import moss_delay as O
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libmtts.so not built")
    D, n = 16, 512
    cs = np.zeros((n, D), np.uint16)
    sn = np.zeros((n, D), np.uint16)
    _native.call("mtts_rope_table", ctypes.c_float(1e4), D, n, cs.ctypes.data_as(ctypes.c_void_p),
                 sn.ctypes.data_as(ctypes.c_void_p))
    c, s = O.rope_cos_sin(O._Ctx("bf16"), O.tiny_cfg(), np.arange(n))
    assert np.mean(B16.from_bits(cs) == c) > 0.999 and np.mean(B16.from_bits(sn) == s) > 0.999


def test_build_id_matches_tree():
    """the library's compiled-in source hash is this tree's (moss_tts_amd/_buildid.py); a
    stale prebuilt binary is refused by the binding and by tests/conftest.py"""
    from moss_tts_amd import _buildid, _native
    if not os.path.exists(_native.lib_path()):
        pytest.skip("libmtts.so not built")
    assert _native.build_id() == _buildid.tree_hash("lib")
    assert len(_native.build_id()) == 64
