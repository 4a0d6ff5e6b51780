"""analysis — the reference's src/analysis module, restricted to what runs on the alignment hot
path (seq::edit_distance)."""
from . import seq  # noqa: F401
