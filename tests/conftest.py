import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# torch ships its own HIP runtime (torch/lib/libamdhip64.so) and the library binds to whichever
# libamdhip64 the process loaded first: import torch before any test loads libbiogarden_gpu.so,
# or a later torch.cuda call finds no GPU (two runtimes in one process).  Importing initialises
# no device.
try:
    import torch  # noqa: F401
except ImportError:
    pass

GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_FIX = os.path.join(GOLDEN, "reference_fixtures")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libbiogarden_gpu.so)")


def read_fasta(path):
    """Minimal independent FASTA parse for fixtures (the product reader is tested against it)."""
    recs = []
    with open(path) as f:
        for line in f:
            if line.startswith(">"):
                recs.append([line[1:].split()[0], []])
            elif recs:
                recs[-1][1].append(line.rstrip())
    return [(r[0], "".join(r[1]).encode()) for r in recs]


# The reference's alignment integration tests (tests/integration.rs:234-312):
# (mode, scoring, open, extend, expected score)
REFERENCE_GOLDENS = [
    ("global", "blosum62", -11, -1, 232),
    ("local", "blosum62", -11, -1, 20431),
    ("fitting", "unit", -1, -1, 145),
    ("overlap", "unit", -2, -2, 698),
    ("semiglobal", "unit", -1, -1, 982),
]

# The aligner doctests (aligner.rs:68-83, 134-149, 198-215, 273-289, 336-350)
REFERENCE_DOCTESTS = [
    ("global", b"PRTEINS", b"PRTWPSEIN", "blosum62", -11, -1, 8, b"PRT---EINS", b"PRTWPSEIN-"),
    ("local", b"PLEASANTLY", b"MEANLY", "blosum62", -11, -1, 12, b"LEAS", b"MEAN"),
    ("fitting",
     b"GCAAACCATAAGCCCTACGTGCCGCCTGTTTAAACTCGCGAACTGAATCTTCTGCTTCACGGTGAAAGTACCACAATGGTATCACACCCCAAGGAAAC",
     b"GCCGTCAGGCTGGTGTCCG", "unit", -1, -1, 5, b"GCCCT-A--C-G-TG-CCG", b"GCCGTCAGGCTGGTGTCCG"),
    ("overlap", b"CTAAGGGATTCCGGTAATTAGACAG", b"ATAGACCATATGTCAGTGACTGTGTAA", "unit", -2, -2, 2,
     b"ATTAGAC-AG", b"AT-AGACCAT"),
    ("semiglobal", b"TAGCACTTGGATTCTCGG", b"CAGCGTGG", "unit", -1, -1, 4,
     b"TAGCA-CTTGGATTCTCGG", b"---CAGCGTGG--------"),
]


@pytest.fixture(scope="session")
def oracle():
    from oracle import refcpu
    refcpu.lib()
    return refcpu
