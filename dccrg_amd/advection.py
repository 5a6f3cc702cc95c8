"""The advection test program of the reference (tests/advection/2d.cpp with
initialize.hpp, solve.hpp and adapter.hpp) over the device grid: the
per-step solver and the neighbor-difference adaptation run as HIP kernels
(dccrgx_advect_step, dccrgx_advect_adapt_marks); the refinement decisions
and the data handed to new cells follow adapter.hpp on the host, as the
reference does.

Geometry: tests/advection/2d.cpp:200-250 for direction 'z' -- a Cartesian
geometry starting at 0 with level-0 cell length 1 / cells along every axis
(z included, :241-243).
"""
from __future__ import annotations

import ctypes as C
from typing import Tuple

import numpy as np

from . import _capi as X
from ._capi import check, lib
from .grid import Dccrg


class CartesianGeometry:
    """Cartesian_Geometry (dccrg_cartesian_geometry.hpp) for the cell
    centers and lengths the advection program needs."""

    def __init__(self, grid: Dccrg, start=(0.0, 0.0, 0.0), level_0_cell_length=None):
        self.grid = grid
        self.start = np.asarray(start, dtype=np.float64)
        n = np.asarray(grid._length, dtype=np.float64)
        self.l0 = np.asarray(level_0_cell_length if level_0_cell_length is not None else 1.0 / n,
                             dtype=np.float64)

    def centers_and_lengths(self, cells: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        m = self.grid.mapping
        M = m.max_ref_lvl
        idx, lvl = m.levels_and_indices(cells)
        idx = idx.astype(np.float64)
        ln = self.l0[None, :] / (2.0 ** lvl.astype(np.float64))[:, None]
        center = self.start[None, :] + idx * (self.l0 / 2.0 ** M)[None, :] + ln / 2
        return center, ln


def geometry_2d(grid: Dccrg) -> CartesianGeometry:
    """2d.cpp:238-243 (direction 'z'): start 0, level-0 cell length
    GRID_END / cells = 1 / cells along x, y and z."""
    cells = grid._length[0]
    return CartesianGeometry(grid, (0.0, 0.0, 0.0), [1.0 / cells] * 3)


def get_vx(y):  # solve.hpp:336-338
    return -y + 0.5


def get_vy(x):  # solve.hpp:340-342
    return x - 0.5


ALL = ("density", "flux", "vx", "vy", "vz", "length_x", "length_y", "length_z")


def initialize(grid: Dccrg, geom: CartesianGeometry, update: bool = True):
    """initialize.hpp:27-65: hump density, solid-body velocities, lengths.
    update=False leaves the final ghost update (:60) to the caller (ranks
    driven in one process exchange through pack / unpack)."""
    cells = grid.local_cells()
    center, ln = geom.centers_and_lengths(cells)
    r = np.minimum(np.sqrt((center[:, 0] - 0.25) ** 2 + (center[:, 1] - 0.5) ** 2), 0.15) / 0.15
    grid.write_local("density", 0.25 * (1 + np.cos(np.pi * r)))
    grid.write_local("flux", np.zeros(cells.size))
    _velocities_lengths(grid, geom)
    if update:
        grid.update_copies_of_remote_neighbors(fields=list(ALL))


def _velocities_lengths(grid, geom, cells=None, center=None, ln=None):
    """adapter.hpp:304-314 / initialize.hpp:50-58 on the device
    (dccrgx_advect_set_geometry: get_center / get_length of every local cell
    from its id, then the solid-body velocities)."""
    f = grid._advect_fields()
    start = (C.c_double * 3)(*[float(v) for v in geom.start])
    l0 = (C.c_double * 3)(*[float(v) for v in geom.l0])
    check(lib().dccrgx_advect_set_geometry(grid._h, C.byref(f), start, l0))


def check_for_adaptation(grid: Dccrg, diff_increase: float, diff_threshold: float,
                         unrefine_sensitivity: float):
    """adapter.hpp:43-176 on the device (dccrgx_advect_adaptation_sets): the
    differences, categories and the per-sibling-group rules of :120-175
    (their outcome does not depend on the order the reference visits cells
    in).  Returns (cells_to_refine, cells_not_to_unrefine, cells_to_unrefine),
    each ascending."""
    empty = np.zeros(0, dtype=np.uint64)
    if grid.get_maximum_refinement_level() == 0:
        return empty, empty, empty
    n = grid.n_local
    out = [np.empty(max(n, 1), dtype=np.uint64) for _ in range(3)]
    counts = (C.c_size_t * 3)()
    f = grid._advect_fields()
    check(lib().dccrgx_advect_adaptation_sets(grid._h, X.DEFAULT_NEIGHBORHOOD_ID, C.byref(f), diff_increase,
                                              diff_threshold, unrefine_sensitivity,
                                              *[a.ctypes.data_as(X._u64p) for a in out], max(n, 1), counts))
    grid._refresh_info()
    return tuple(a[:k].copy() for a, k in zip(out, counts))


def check_and_request(grid: Dccrg, diff_increase: float, diff_threshold: float,
                      unrefine_sensitivity: float) -> Tuple[int, int, int]:
    """check_for_adaptation followed by request_adaptation with the three
    sets kept on the device (dccrgx_advect_adapt_requests): the same request
    state, without the sets' round trip through host memory.  The requests
    read only the leaf structure, not the density, so they may be made before
    the solver step that 2d.cpp runs between the check and adapt_grid; finish
    with finish_adaptation.  Returns the three set sizes."""
    if grid.get_maximum_refinement_level() == 0:
        return 0, 0, 0
    counts = (C.c_size_t * 3)()
    f = grid._advect_fields()
    check(lib().dccrgx_advect_adapt_requests(grid._h, X.DEFAULT_NEIGHBORHOOD_ID, C.byref(f), diff_increase,
                                             diff_threshold, unrefine_sensitivity, counts))
    grid._refresh_info()
    return tuple(int(c) for c in counts)


def _request(grid: Dccrg, kind: int, ids: np.ndarray):
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    check(lib().dccrgx_amr_request_cells(grid._h, kind, ids.ctypes.data_as(X._u64p), ids.size, None))


def adapt_grid(grid: Dccrg, geom: CartesianGeometry, to_refine, not_to_unrefine, to_unrefine,
               all_requests=None) -> Tuple[int, int]:
    """adapter.hpp:184-319.  Returns (created, removed) cell counts."""
    if grid.get_maximum_refinement_level() == 0:
        return 0, 0
    request_adaptation(grid, to_refine, not_to_unrefine, to_unrefine)
    return finish_adaptation(grid, geom, all_requests)


def request_adaptation(grid: Dccrg, to_refine, not_to_unrefine, to_unrefine):
    """adapter.hpp:197-213: this rank's requests (before the collective
    stop_refining)."""
    if grid.get_maximum_refinement_level() == 0:
        return
    _request(grid, X.AMR_REFINE, to_refine)
    _request(grid, X.AMR_DONT_UNREFINE, not_to_unrefine)
    _request(grid, X.AMR_UNREFINE, to_unrefine)
    grid._refresh_info()


def finish_adaptation(grid: Dccrg, geom: CartesianGeometry, all_requests=None,
                      update: bool = True) -> Tuple[int, int]:
    """adapter.hpp:215-319: stop_refining (all_requests: the union of every
    rank's requests), data of new cells and of the parents of removed cells,
    velocities and lengths, ghost update (skipped with update=False)."""
    if grid.get_maximum_refinement_level() == 0:
        return 0, 0
    if grid.ctx.comm_size == 1 and all_requests is None:
        n_new = grid.stop_refining_count()  # the new cells' count only (no copy of the list)
    else:
        n_new = grid.stop_refining(all_requests=all_requests).size
    return _after_stop_refining(grid, geom, n_new, update)


def finish_adaptation_all(grids, geoms, all_requests, update: bool = False):
    """finish_adaptation of several ranks held in one process: the
    collective stop_refining across them (stop_refining_all: all adopt the new
    grid or all keep the old one), then each rank's data rules."""
    from .grid import stop_refining_all
    if grids[0].get_maximum_refinement_level() == 0:
        return [(0, 0) for _ in grids]
    news = stop_refining_all(grids, all_requests)
    return [_after_stop_refining(g, geom, new.size, update) for g, geom, new in zip(grids, geoms, news)]


def _after_stop_refining(grid: Dccrg, geom: CartesianGeometry, n_new: int, update: bool) -> Tuple[int, int]:
    n_removed = C.c_size_t()
    check(lib().dccrgx_get_removed_cells(grid._h, None, 0, C.byref(n_removed)))
    # new cells are value-initialised by the rebuild (flux = 0); they take the
    # parent's density (:229-251).  Parents of removed cells: 0, then
    # += child / 8 over the children in ascending order (:253-300).  Both on
    # the device, from the retired cells' data, in one call.
    fd = getattr(grid, "_adv_density_fid", None)
    if fd is None:
        fd = grid._adv_density_fid = np.array([grid.field_id("density")], dtype=np.int32)
    check(lib().dccrgx_amr_adapter_data_rules(grid._h, fd.ctypes.data_as(X._i32p), fd.size))
    grid.clear_refined_unrefined_data()
    # velocities and lengths of every local cell (:303-313)
    _velocities_lengths(grid, geom)
    if update:
        grid.update_copies_of_remote_neighbors(fields=list(ALL))
    return int(n_new), int(n_removed.value)


def max_time_step(grid: Dccrg) -> float:
    """solve.hpp:302-332 on one rank (the caller reduces with MIN)."""
    return grid.max_time_step()
