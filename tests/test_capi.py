"""The C-ABI library builds, loads and exports every symbol include/gossip_capi.h
declares; error behaviour without a GPU (no compute calls here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "gossip_capi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gp_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_the_binding(pkg):
    decl = declared_symbols()
    assert set(decl) == set(pkg._lib.SIGNATURES), set(decl) ^ set(pkg._lib.SIGNATURES)


def test_library_exports_every_symbol(pkg):
    lib = pkg._lib.load()
    raw = ctypes.CDLL(pkg._lib.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(raw, name), name
    assert lib.gp_abi_version() == pkg._lib.ABI_VERSION == 12


def test_no_gpu_is_an_error_not_a_fallback(pkg):
    lib = pkg._lib.load()
    if pkg._lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(pkg.GossipError):
        pkg.GossipEngine(0)
    cfg = pkg._lib.Config()
    lib.gp_default_config(ctypes.byref(cfg))
    assert cfg.miss_threshold == 3 and cfg.hub_threshold >= 64
    assert lib.gp_round(None, None) == pkg._lib.GP_EINVAL
    assert b"null" in lib.gp_last_error()


def test_missing_library_fails_loudly(pkg, tmp_path, monkeypatch):
    import importlib
    lib_mod = importlib.import_module("gossip_amd._lib")
    monkeypatch.setattr(lib_mod, "_lib", None)
    with pytest.raises(lib_mod.GossipLibraryError):
        lib_mod.load(str(tmp_path / "nope.so"))
