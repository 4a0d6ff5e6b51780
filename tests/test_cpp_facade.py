"""The C++ host facade (include/biogarden.hpp) over the C ABI: compiled with g++ against the
in-tree libbiogarden_gpu.so.  CPU part here; the reference's integration goldens through the
facade on the GPU in test_cpp_integration."""
import os
import subprocess

import pytest

from conftest import ROOT, REF_FIX

LIB_DIR = os.path.join(ROOT, "biogarden_amd")


def build(src, out):
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", src), "-L", LIB_DIR, "-lbiogarden_gpu",
           "-Wl,-rpath," + LIB_DIR, "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return str(out)


def test_facade_cpu(tmp_path):
    exe = build("test_facade.cpp", tmp_path / "test_facade")
    args = [exe, REF_FIX]
    import torch
    if not torch.cuda.is_available():
        args.append("--no-gpu")
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "facade ok" in r.stdout


@pytest.mark.gpu
def test_facade_integration_goldens(tmp_path):
    """tests/integration.rs:234-312 through biogarden::alignment::SequenceAligner."""
    exe = build("test_integration.cpp", tmp_path / "test_integration")
    r = subprocess.run([exe, REF_FIX], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "integration ok" in r.stdout
