from . import aligner, score  # noqa: F401
