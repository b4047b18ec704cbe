"""dltb.ops — kernel-level ops.

``functional`` dispatches GPU tensors to the gfx950 HIP kernels of ``dltb._C`` and CPU tensors to
the torch references in ``ref``; ``rng`` is the shared counter-hash dropout RNG.
"""
from . import functional, ref, rng  # noqa: F401
from ._ext import available as ext_available, ext  # noqa: F401
