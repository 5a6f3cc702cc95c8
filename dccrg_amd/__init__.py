"""dccrg_amd -- MI355X-native hot path of dccrg (cell-id mapping, neighbor
lists, stencil iteration, remote-neighbor halo exchange).

The compute lives in libdccrgx.so (HIP, gfx950); this package is the host
mirror of the reference interface over its C-ABI (include/dccrgx.h).
"""
from ._capi import (DEFAULT_NEIGHBORHOOD_ID, ERROR_CELL, ERROR_INDEX, DccrgxError,  # noqa: F401
                    LIB_PATH, lib)
from .grid import Context, Dccrg, Mapping, cartesian_geometry, no_geometry, stop_refining_all  # noqa: F401
from .poisson import PoissonSolve  # noqa: F401

__all__ = ["Context", "Dccrg", "Mapping", "DccrgxError", "DEFAULT_NEIGHBORHOOD_ID", "ERROR_CELL",
           "ERROR_INDEX", "LIB_PATH", "lib", "PoissonSolve", "cartesian_geometry", "no_geometry", "stop_refining_all"]
