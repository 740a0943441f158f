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
