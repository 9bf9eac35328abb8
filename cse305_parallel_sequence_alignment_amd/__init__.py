"""MI355X-native pairwise sequence alignment (hot path of D-2n/CSE305_Parallel_Sequence_Alignment).

Native pieces: ``libmsa.so`` (HIP kernels for gfx950 + the C-ABI in
``include/msa.h``).  Python here is a thin mirror of the reference's C++
interface (see ``api``) plus device-resident plans for batch work (``plan``).
"""
from . import _lib
from ._lib import MsaError

__all__ = ["MsaError", "_lib"]
