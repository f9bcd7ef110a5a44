"""singa_amd -- an MI355X-native (gfx950 / CDNA4) deep-learning framework with
the capabilities of ug93tad/singa plus the later Apache SINGA Python API.

Import order matters: torch is imported first so the HIP runtime torch ships
(libamdhip64.so.7) is the one the gfx950 kernel library binds to.
"""
import torch  # noqa: F401  (must precede the native modules)

from . import device, tensor, autograd, layer, model, opt  # noqa: F401
from .ops import native as _native  # noqa: F401

__version__ = "0.1.0"


def native_loaded() -> bool:
    return _native.available()


def set_deterministic(on: bool = True) -> None:
    """Deterministic mode: ordered (atomic-free) BatchNorm and
    fused-statistics reductions and single-split weight gradients, so a
    training step is bitwise reproducible run to run (slower).  Philox
    dropout streams are already reproducible for a given device seed."""
    if _native.available():
        _native.lib().set_deterministic(int(bool(on)))
    import os

    os.environ["SINGA_AMD_DETERMINISTIC"] = "1" if on else "0"
