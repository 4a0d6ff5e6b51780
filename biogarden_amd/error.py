"""Errors — mirrors src/error.rs:8-14 (BioError) of the reference crate.

The reference returns `Err(BioError::InvalidArgumentRange | InvalidInputSize)` from the aligner
and *panics* on unscorable bytes / out-of-range buffer indices; here a panic of the reference
is surfaced as ReferencePanic so callers can tell the two apart.
"""


class BioError(Exception):
    """Base of the reference's error variants."""


class InvalidInputSize(BioError):
    """BioError::InvalidInputSize — "Provided inputs have invalid size!" (error.rs:19)."""


class InvalidArgumentRange(BioError):
    """BioError::InvalidArgumentRange (error.rs:20)."""


class ItemNotFound(BioError):
    pass


class TypeConversionError(BioError):
    pass


class ReferencePanic(RuntimeError):
    """The reference implementation would panic (or hang) on this input; `result` holds the
    exactly-sized DP's answer when one exists (DESIGN.md "Buffer semantics")."""

    def __init__(self, msg, result=None):
        super().__init__(msg)
        self.result = result
