"""AddressSanitizer + UBSan builds of the host code, CPU only:

* the host byte passes of bg_batch_prepare / bg_batch_fetch (biogarden_amd/csrc/bg_host_passes.h:
  validation and staging, code sets, the scratch history, string unpacking, the worker pool)
  against restatements on random batches (tests/cpp/test_host_passes.cpp);
* the native FASTA batch reader (biogarden_amd/csrc/bg_fasta.cpp) on the reference fixtures and
  adversarial files at 1-byte to 4-MiB blocks, compared with the Python mirror of fasta.rs;
* the CPU oracle (oracle/refcpu.c), test infrastructure itself, on random pairs through a reused
  reference-faithful aligner (resizes, panics) and exact-size ones.

Each binary is built with g++ / gcc -fsanitize=address,undefined -fno-sanitize-recover=all; a
sanitizer report fails the run."""
import glob
import os
import random
import subprocess

import pytest

from conftest import REF_FIX, ROOT

SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
       "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
           UBSAN_OPTIONS="print_stacktrace=1")


def _build(tmp_path, name, cmd):
    exe = str(tmp_path / name)
    r = subprocess.run(cmd + ["-o", exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def _run(args, timeout=300):
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=ENV)
    assert r.returncode == 0 and "ERROR: AddressSanitizer" not in r.stderr and \
        "runtime error" not in r.stderr, (r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


def test_host_passes_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "host_passes", ["g++", "-std=c++17", "-pthread", "-I",
                                           os.path.join(ROOT, "include")] + SAN +
                 [os.path.join(ROOT, "tests", "cpp", "test_host_passes.cpp")])
    assert "host passes ok" in _run([exe])


def test_oracle_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "oracle_fuzz", ["gcc", "-std=c11", "-D_POSIX_C_SOURCE=200809L",
                                           "-pthread"] + SAN +
                 [os.path.join(ROOT, "tests", "cpp", "test_oracle_fuzz.c"),
                  os.path.join(ROOT, "oracle", "refcpu.c")])
    assert "oracle fuzz ok" in _run([exe], timeout=600)


def _py_dump(path):
    from biogarden_amd.io import fasta
    try:
        r = fasta.Reader.from_file(path)
        try:
            recs = list(r.records())
        finally:
            r.close()
    except IOError as e:
        return "ERR " + str(e)
    return "".join("%s\t%s\t%s\n" % (x.id(), "-" if x.desc() is None else x.desc(),
                                      x.seq().decode("utf-8", "surrogateescape")) for x in recs)


@pytest.fixture(scope="module")
def fasta_exe(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("fasta")
    return _build(tmp, "fasta_dump", ["g++", "-std=c++17", "-I", os.path.join(ROOT, "include")] + SAN +
                  [os.path.join(ROOT, "tests", "cpp", "test_fasta_dump.cpp"),
                   os.path.join(ROOT, "biogarden_amd", "csrc", "bg_fasta.cpp")])


def _files(tmp_path):
    files = sorted(glob.glob(os.path.join(REF_FIX, "input", "*.fasta")))
    rng = random.Random(4)
    for k in range(6):
        lines = []
        for r in range(rng.randint(1, 30)):
            lines.append(">" + "".join(rng.choice("ab c\t") for _ in range(rng.randint(0, 9))) +
                         rng.choice(["", " ", "\r"]))
            for _ in range(rng.choice([0, 1, 3])):
                lines.append("".join(rng.choice("ACGT") for _ in range(rng.choice([0, 1, 60, 300]))) +
                             rng.choice(["", " ", "\r", "　"]))
        p = tmp_path / ("g%d.fa" % k)
        p.write_bytes(("\n".join(lines) + rng.choice(["", "\n"])).encode("utf-8"))
        files.append(str(p))
    for k, data in enumerate([b"", b">", b"ACGT\n", b">a\nAC\xffGT\n", b">a\xc3", b">a\n\n\n>b\nC",
                              b">x\n>\n>y\nG\n"]):
        p = tmp_path / ("e%d.fa" % k)
        p.write_bytes(data)
        files.append(str(p))
    return files


@pytest.mark.parametrize("block", ["1", "7", "4194304"])
def test_fasta_reader_asan_ubsan(tmp_path, fasta_exe, block):
    for path in _files(tmp_path):
        want = _py_dump(path)
        for maxr, maxres in (("1", "1000000000"), ("3", "100"), ("100000", "1")):
            env_block = dict(ENV, BG_FASTA_BLOCK=block)
            r = subprocess.run([fasta_exe, path, maxr, maxres], capture_output=True, timeout=120,
                               env=env_block)
            assert r.returncode == 0 and b"runtime error" not in r.stderr and \
                b"AddressSanitizer" not in r.stderr, r.stderr[-3000:]
            got = r.stdout.decode("utf-8", "surrogateescape")
            if want.startswith("ERR"):
                assert "ERR -8" in got or "ERR -9" in got, (path, got)
                assert ("ERR -9" in got) == ("UTF-8" in want), (path, got, want)
            else:
                assert got == want, (path, block, maxr, maxres)
