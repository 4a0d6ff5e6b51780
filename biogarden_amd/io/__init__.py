from . import fasta  # noqa: F401
