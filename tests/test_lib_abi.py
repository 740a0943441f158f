"""CPU checks of the C-ABI library: it loads, exports every symbol the public
header declares, and fails loudly (no CPU fallback) where there is no GPU."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "flamingo_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(flm_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from flamingo_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from flamingo_amd import build
        build.build()
    return _lib.load()


def test_exports_every_header_symbol(lib):
    syms = header_symbols()
    assert len(syms) >= 19
    for s in syms:
        assert hasattr(lib, s), s


def test_python_binding_covers_header(lib):
    from flamingo_amd import _lib
    assert set(header_symbols()) == set(_lib.SIGNATURES)


def test_version_and_no_silent_fallback(lib):
    assert b"gfx950" in lib.flm_version()
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    ctx = ctypes.c_void_p()
    rc = lib.flm_init(ctypes.byref(ctx), 0)
    assert rc != 0 and not ctx.value
    assert lib.flm_last_error(None)
    from flamingo_amd import MaskEngine
    with pytest.raises(RuntimeError):
        MaskEngine(0)


def test_gfx950_code_object(lib):
    from flamingo_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"items_kernel" in data


def test_round5_entry_points_reject_null_handles(lib):
    """flm_comm_destroy, flm_hash_to_curve*, flm_store_unmask_ms: a NULL context / store is an
    FLM_EINVAL with a message, before any device call (no GPU needed)."""
    buf = (ctypes.c_uint8 * 64)()
    fl = (ctypes.c_uint32 * 1)()
    ln = (ctypes.c_uint32 * 1)(3)
    assert lib.flm_comm_destroy(None) == -1 and b"NULL" in lib.flm_last_error(None)
    assert lib.flm_hash_to_curve(None, buf, ln, 1, buf, fl) == -1
    assert lib.flm_hash_to_curve_decimal(None, 0, 1, buf, fl) == -1
    assert lib.flm_hash_to_curve_decimal_dev(None, 0, 1, None, None, None) == -1
    ms = ctypes.c_float()
    assert lib.flm_store_unmask_ms(None, ctypes.byref(ms)) == -1
    assert b"0.4" in lib.flm_version()


def test_round6_entry_points_reject_null_handles(lib):
    """flm_get_tuning (round 6): a NULL context, key or output is an FLM_EINVAL with a message,
    before any device call; the expansion knobs are refused on a NULL context too."""
    v = ctypes.c_int(7)
    assert lib.flm_get_tuning(None, b"pairing", ctypes.byref(v)) == -1 and b"NULL" in lib.flm_last_error(None)
    assert v.value == 7
    assert lib.flm_set_tuning(None, b"expand_waves", 8) == -1
