"""Poisson_Solve (tests/poisson/poisson_solve.hpp:138-1057) on the device.

Mirrors the reference class: construct with the solver parameters, then
``solve(cells, cells_to_skip, cache_is_up_to_date)``.  Cell data lives in the
grid's f64 fields: the user's rhs / solution / cell lengths and the solver's
own members (registered on the grid as ``poisson.<member>``).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi as X
from ._capi import check, lib


class PoissonSolve:
    def __init__(self, grid, max_iterations: int = 1000, min_iterations: int = 0,
                 stop_residual: float = 1e-15, p_of_norm: float = 2.0,
                 stop_after_residual_increase: float = 10.0, fields=None):
        names = {"rhs": "rhs", "solution": "solution", "length_x": "length_x", "length_y": "length_y",
                 "length_z": "length_z"}
        names.update(fields or {})
        self.grid = grid
        prm = X.PoissonParams_t(max_iterations, min_iterations, stop_residual, p_of_norm,
                                stop_after_residual_increase)
        f = X.PoissonFields_t(*[grid.field_id(names[k]) for k in ("rhs", "solution", "length_x", "length_y",
                                                                    "length_z")])
        h = C.c_void_p()
        check(lib().dccrgx_poisson_create(grid._h, C.byref(prm), C.byref(f), C.byref(h)))
        self._h = h.value
        for i, m in enumerate(X.POISSON_MEMBERS):
            fid = C.c_int32()
            check(lib().dccrgx_poisson_field(self._h, i, C.byref(fid)))
            grid._fields["poisson." + m] = (fid.value, np.dtype(np.float64))

    def solve(self, cells, cells_to_skip=(), cache_is_up_to_date: bool = False):
        """Returns (iterations, minimum residual)."""
        c = np.ascontiguousarray(cells, dtype=np.uint64)
        s = np.ascontiguousarray(cells_to_skip, dtype=np.uint64)
        it = C.c_uint32()
        res = C.c_double()
        check(lib().dccrgx_poisson_solve(self._h, c.ctypes.data_as(X._u64p), c.size, s.ctypes.data_as(X._u64p),
                                         s.size, int(cache_is_up_to_date), C.byref(it), C.byref(res)))
        return it.value, res.value

    def close(self):
        if getattr(self, "_h", None):
            lib().dccrgx_poisson_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
