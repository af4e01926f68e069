"""arcanefem_amd — MI355X-native FEM global-matrix assembly + Jacobi-PCG path.

A drop-in for the DoFLinearSystem / IDoFLinearSystemFactory / BSRFormat
surface of toutane/arcanefem (femutils/), implemented as hand-written HIP for
gfx950 behind the C ABI of include/arcanefem_amd.h (libafem.so, in-tree).
"""
from ._capi import AfemError, LIB_PATH, load  # noqa: F401
from .core import (BSRFormat, Communicator, Context, DoFLinearSystem, HipDoFLinearSystemFactory,  # noqa: F401
                   Mesh, applyNeumannToRhs, device_count, partition_rcb, set_variant, structured_halo_plan,
                   subdomain_plan)

__version__ = "0.1.0"
