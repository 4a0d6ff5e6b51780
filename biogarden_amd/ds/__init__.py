from .sequence import Sequence  # noqa: F401
from .tile import Tile  # noqa: F401
