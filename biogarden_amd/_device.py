"""The process-wide default GPU handle used by the reference's free functions
(analysis::seq::edit_distance, processing::patterns::*), created on first use on device 0."""
from . import _native

_HANDLE = None


def handle():
    global _HANDLE
    if _HANDLE is None:
        _HANDLE = _native.Handle(0)
    return _HANDLE
