"""Mirror of the reference's `src/core` drivers on the SBA / FTE path (src/core/__init__.py)."""
from .tri import tri  # noqa: F401
from .sba import sba  # noqa: F401
from .fte import fte  # noqa: F401
from .ekf import ekf  # noqa: F401
