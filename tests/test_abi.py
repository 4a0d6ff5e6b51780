"""The C-ABI library: loads, exports every symbol include/biogarden_gpu.h declares, and its
host-only entry points behave without a GPU.  No compute calls here."""
import ctypes
import os
import re

from conftest import ROOT


def declared_functions():
    with open(os.path.join(ROOT, "include", "biogarden_gpu.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bg_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from biogarden_amd import _native
    L = _native.lib()
    decl = declared_functions()
    assert len(decl) >= 13
    missing = [s for s in decl if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(_native.EXPORTS) == decl


def test_host_only_entry_points():
    from biogarden_amd import _native
    L = _native.lib()
    assert L.bg_abi_version() == 2
    assert L.bg_status_string(0) == b"ok"
    assert L.bg_status_string(1) == b"InvalidArgumentRange"
    sc = _native.BgScoring()
    assert L.bg_scoring_builtin(7, ctypes.byref(sc)) < 0


def test_no_gpu_means_loud_failure():
    import torch
    if torch.cuda.is_available():
        return
    from biogarden_amd import _native
    try:
        _native.Handle(0)
    except _native.NativeUnavailable:
        return
    raise AssertionError("bg_aligner_new succeeded without a GPU")


def test_missing_library_is_loud(monkeypatch, tmp_path):
    """No CPU fallback: an unbuilt library raises NativeUnavailable before any compute."""
    from biogarden_amd import _native
    monkeypatch.setattr(_native, "_LIB", None)
    monkeypatch.setattr(_native, "LIB_PATH", str(tmp_path / "libbiogarden_gpu.so"))
    try:
        _native.lib()
    except _native.NativeUnavailable:
        return
    raise AssertionError("lib() loaded without the built library")


def test_library_is_gfx950():
    """The shipped code object targets gfx950 only (no multi-arch / CUDA shims)."""
    path = os.path.join(ROOT, "biogarden_amd", "libbiogarden_gpu.so")
    data = open(path, "rb").read()
    assert b"gfx950" in data
    assert b"sm_" not in data.split(b"gfx950")[0][-64:]
