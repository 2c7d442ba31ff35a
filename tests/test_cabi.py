"""The C-ABI library loads and exports every symbol include/ptv_api.h declares
(CPU only: no compute call needs a GPU here)."""
import ctypes
import os
import re

import pytest

from ptv_interpolation_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    src = open(os.path.join(ROOT, "include", "ptv_api.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ptv_[a-z0-9_]+)\s*\(", src)))


def test_library_present_and_loads():
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() first"
    _lib.lib()


def test_every_declared_symbol_is_exported():
    names = _header_functions()
    assert "ptv_interp_knn" in names and "ptv_init" in names
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the Python binding covers all of them
    assert set(names) <= set(_lib.EXPORTS), set(names) - set(_lib.EXPORTS)


def test_version_matches_header():
    src = open(os.path.join(ROOT, "include", "ptv_api.h")).read()
    v = int(re.search(r"#define PTV_API_VERSION (\d+)", src).group(1))
    assert _lib.lib().ptv_version() == v


def test_struct_layouts_agree():
    c, py = _lib.abi_sizes()
    assert c == py
    c2, py2 = _lib.abi_sizes2()
    assert c2 == py2
    c3, py3 = _lib.abi_sizes3()
    assert c3 == py3


def test_no_gpu_fails_loudly():
    """Without a visible GPU the context refuses to start (no silent CPU fallback)."""
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises((ValueError, _lib.PtvError), match="device"):
        _lib.Context(0)


def test_error_codes_map_to_exceptions():
    with pytest.raises(ValueError):
        _lib.check(_lib.PTV_E_ARG)
    with pytest.raises(NotImplementedError):
        _lib.check(_lib.PTV_E_UNSUPPORTED)
    with pytest.raises(MemoryError):
        _lib.check(_lib.PTV_E_NOMEM)
