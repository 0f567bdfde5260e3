"""ccmpc -- MI355X-native Monte-Carlo prediction + MVOE chance-constraint path of CC-MPC.

Host mirror of the reference planner's constraint-generation surface (v8ideal) over the
C ABI of libccmpc.so (include/ccmpc.h).  GPU only: there is no CPU fallback.
"""
from . import _lib, risk  # noqa: F401
from ._lib import CcmpcError, HALFSPACE_DTYPE, AFFINE_DTYPE  # noqa: F401

__all__ = ["CcmpcError", "HALFSPACE_DTYPE", "AFFINE_DTYPE", "risk"]
