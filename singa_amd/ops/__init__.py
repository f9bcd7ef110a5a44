"""Op layer: native gfx950 kernels (GPU) and PyTorch reference (CPU)."""
from . import native  # noqa: F401
from . import functional  # noqa: F401
from .functional import *  # noqa: F401,F403
