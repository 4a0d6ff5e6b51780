"""biogarden_amd — MI355X-native drop-in for robsndr/biogarden's pairwise-alignment hot path.

Module layout mirrors the reference crate (src/lib.rs): alignment.{aligner,score},
ds.{sequence,tile}, io.fasta, error.  The compute runs in libbiogarden_gpu.so (HIP, gfx950).
"""
__version__ = "0.1.0"

from . import error  # noqa: F401
from .ds import Sequence, Tile  # noqa: F401
