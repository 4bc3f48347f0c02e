"""The C-ABI library loads and exports every symbol include/csa_legacy.h declares (no GPU calls)."""
import ctypes
import re

from conftest import pkg


def _declared():
    N = pkg("_native")
    with open(N.HEADER) as fh:
        text = fh.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(csa_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    N = pkg("_native")
    L = N.lib()
    declared = _declared()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(L, name), name
        assert name in N.SIGNATURES, "ctypes signature missing for " + name
    assert set(N.SIGNATURES) == set(declared)


def test_version_and_error_plumbing():
    N = pkg("_native")
    L = N.lib()
    assert L.csa_version() == 1
    # invalid arguments are rejected on the host without touching a device
    h = ctypes.c_void_p()
    rc = L.csa_instance_create(-1, 0, 0, None, None, None, None, ctypes.byref(h))
    assert rc == N.CSA_E_INVALID
    assert "invalid" in N.last_error()
    assert L.csa_xt_pad(1) == 256 and L.csa_xt_pad(1727) == 1792 and L.csa_xt_pad(2000) == 2048


def test_no_cpu_fallback_when_library_missing(monkeypatch, tmp_path):
    N = pkg("_native")
    monkeypatch.setattr(N, "_lib", None)
    monkeypatch.setattr(N, "LIB_PATH", str(tmp_path / "missing.so"))
    try:
        N.lib()
    except N.NativeLibraryError as e:
        assert "no CPU fallback" in str(e)
    else:
        raise AssertionError("missing library must raise")
