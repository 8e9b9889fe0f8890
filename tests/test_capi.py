"""The C-ABI library builds, loads and exports every symbol include/gossip_capi.h
declares; the binding's structs and the INTEGRATION.md stub have the header's
layouts; error behaviour without a GPU (no compute calls here)."""
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
    assert lib.gp_abi_version() == pkg._lib.ABI_VERSION == 18


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


_CTYPES = {"int32_t": ctypes.c_int32, "uint32_t": ctypes.c_uint32, "int64_t": ctypes.c_int64,
           "uint64_t": ctypes.c_uint64, "double": ctypes.c_double, "uint8_t": ctypes.c_uint8}


def header_struct(name):
    """ctypes twin of `typedef struct <name> {...} <name>;` in the header, built
    from its field declarations (ctypes applies the C layout rules)."""
    src = open(os.path.join(ROOT, "include", "gossip_capi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), src, flags=re.S).group(1)
    fields = [(f, _CTYPES[t]) for t, f in re.findall(r"\b(\w+)\s+(\w+)\s*;", body)]
    return type(name, (ctypes.Structure,), {"_fields_": fields})


def layout(cls):
    return [(f, getattr(cls, f).offset, ctypes.sizeof(t)) for f, t in cls._fields_], ctypes.sizeof(cls)


@pytest.mark.parametrize("cname,pyname", [("gp_round_stats", "RoundStats"), ("gp_config", "Config"),
                                          ("gp_report", "Report")])
def test_binding_structs_match_header(pkg, cname, pyname):
    assert layout(getattr(pkg._lib, pyname)) == layout(header_struct(cname))


def test_integration_stub_matches_header(pkg):
    """The ctypes stub INTEGRATION.md tells a maintainer to paste next to
    Peer.py: its RoundStats must be the header's gp_round_stats exactly, or
    every gp_round writes past the caller's struct."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = re.search(r"```python\n(.*?)```", doc, flags=re.S).group(1)
    cls_src = re.search(r"(class RoundStats\(ctypes\.Structure\):.*?)\n(?=\S)", block, flags=re.S).group(1)
    ns = {"ctypes": ctypes}
    exec(cls_src, ns)
    stub = ns["RoundStats"]
    assert layout(stub) == layout(header_struct("gp_round_stats"))
    assert layout(stub) == layout(pkg._lib.RoundStats)
