"""MI355X-native distributed fp64 matrix-vector multiplier (row / column / block split).

Drop-in for yaroslav-i-am/MatVec_MPI_Multiplier's hot path; see DESIGN.md. The compute and
communication live in libmatvec_gpu.so (HIP kernels for gfx950 + RCCL), bound here with ctypes.
"""
from ._lib import lib, check, MvgError, IndivisibleError, Shard  # noqa: F401

__all__ = ["lib", "check", "MvgError", "IndivisibleError", "Shard"]
