"""Host-side mirror of the reference interface on this path.

``Dccrg`` keeps the names, argument meaning and error behaviour of
``dccrg::Dccrg<Cell_Data, Geometry>`` (dccrg.hpp:151-7186) for the hot path:
chained configuration setters, ``initialize``, ``local_cells`` /
``inner_cells`` / ``outer_cells`` / ``remote_cells``, ``get_neighbors_of`` /
``get_neighbors_to``, ``add_neighborhood``, the per-peer send / receive lists
and ``update_copies_of_remote_neighbors`` / ``start_`` / ``wait_`` halo calls.
Cell data lives on the device as structure-of-arrays fields (one per
``Cell_Data`` member); the user stencil runs as a device kernel.

Everything here calls libdccrgx.so; no computation happens in Python.
"""
from __future__ import annotations

import ctypes as C
import struct
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _capi as X
from ._capi import check, lib

DEFAULT_NEIGHBORHOOD_ID = X.DEFAULT_NEIGHBORHOOD_ID


def _dist_ready() -> bool:
    try:
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized()
    except ImportError:
        return False


def set_test_option(name: str, value=None):
    """dccrgx_test_option: force a code path or inject a fault (tests only);
    value None returns the option to its default."""
    check(lib().dccrgx_test_option(name.encode(), 0 if value is None else int(value), 0 if value is None else 1))


class test_option:
    """with test_option("gol_scalar", 1): ... -- set for the block, then reset."""

    def __init__(self, name: str, value):
        self.name, self.value = name, value

    def __enter__(self):
        set_test_option(self.name, self.value)
        return self

    def __exit__(self, *exc):
        set_test_option(self.name, None)
        return False


def stop_refining_all(grids, all_requests):
    """The collective stop_refining of several ranks held in one process (the
    tests' in-process ranks): every grid prepares, then all commit or, when
    any failed, all keep the old grid with the requests pending."""
    res = [g.stop_refining_prepare(all_requests) for g in grids]
    ok = all(st == X.DCCRGX_OK for st, _ in res)
    for g in grids:
        g.stop_refining_finish(ok)
    for st, err in res:
        if st != X.DCCRGX_OK:
            raise X.DccrgxError(st, err)
    return [g.get_new_cells() for g in grids]


class _OnLibraryStream:
    """Stream order between torch and the library without device-wide waits:
    the library's compute stream (as a torch ExternalStream) first waits for
    torch's current stream (the query's input tensors), torch allocates and
    fills the result tensors on it inside the block, the exports run on it
    (stream None), and afterwards torch's current stream waits for it, so the
    results are ordered before whatever the caller queues next.  (torch's
    default stream is the null stream, which the C-ABI cannot name: its NULL
    means the grid's compute stream.)"""

    def __init__(self, ctx, dev):
        import torch
        self.cur = torch.cuda.current_stream(dev)
        self.ls = torch.cuda.ExternalStream(ctx.stream, device=dev)

    def __enter__(self):
        import torch
        self.ls.wait_stream(self.cur)
        self._cm = torch.cuda.stream(self.ls)
        self._cm.__enter__()
        return self

    def __exit__(self, *exc):
        self._cm.__exit__(*exc)
        self.cur.wait_stream(self.ls)
        return False

    def hand_over(self, *tensors):
        """tensors made inside the block and returned to the caller: their
        memory is in use on the caller's stream too (torch's record_stream)"""
        for t in tensors:
            t.record_stream(self.cur)


def _u64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint64)


def no_geometry() -> bytes:
    """No_Geometry's file data (dccrg_no_geometry.hpp:486-549): its id."""
    return struct.pack("<i", 0)


def cartesian_geometry(start, level_0_cell_length) -> bytes:
    """Cartesian_Geometry's file data (dccrg_cartesian_geometry.hpp:620-812)."""
    return struct.pack("<i3d3d", 1, *[float(v) for v in start], *[float(v) for v in level_0_cell_length])


class Context:
    """Device, compute + communication streams, RCCL communicator."""

    def __init__(self, device: int = 0, rank: int = 0, comm_size: int = 1):
        h = C.c_void_p()
        check(lib().dccrgx_ctx_create(device, rank, comm_size, C.byref(h)))
        self._h = h
        self.device, self.rank, self.comm_size = device, rank, comm_size

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(lib().dccrgx_get_unique_id(buf))
        return buf.raw

    def comm_init(self, uid: bytes):
        assert len(uid) == 128
        check(lib().dccrgx_ctx_comm_init(self._h, uid))

    def route_self_through_rccl(self, on: bool = True):
        """Test mode: grids created afterwards send this rank's own periodic
        images through RCCL send/recv to itself (needs comm_init), so the
        multi-rank halo path runs on one GPU."""
        check(lib().dccrgx_ctx_route_self_through_rccl(self._h, 1 if on else 0))

    def synchronize(self):
        check(lib().dccrgx_ctx_synchronize(self._h))

    @property
    def stream(self) -> int:
        s = C.c_void_p()
        check(lib().dccrgx_ctx_compute_stream(self._h, C.byref(s)))
        return s.value or 0

    def close(self):
        if getattr(self, "_h", None):
            lib().dccrgx_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Mapping:
    """dccrg::Mapping (dccrg_mapping.hpp:55-690) with batched device calls.

    Batched methods take / return torch CUDA tensors (device memory plumbing);
    scalar conveniences round-trip one element through the device.
    """

    def __init__(self, length: Sequence[int], max_ref_lvl: int = 0):
        self._m = X.Mapping_t((C.c_uint64 * 3)(*[int(v) for v in length]), int(max_ref_lvl), 0)
        if max_ref_lvl < 0:
            out = C.c_int32()
            check(lib().dccrgx_max_possible_refinement_level(self._m.length, C.byref(out)))
            self._m.max_ref_lvl = out.value
        last = C.c_uint64()
        check(lib().dccrgx_last_cell(C.byref(self._m), C.byref(last)))
        self.last_cell = last.value
        self.length = tuple(int(v) for v in length)

    @property
    def max_ref_lvl(self) -> int:
        return self._m.max_ref_lvl

    def get_maximum_refinement_level(self) -> int:
        return self._m.max_ref_lvl

    def get_last_cell(self) -> int:
        return self.last_cell

    # ---- scalar host calls (dccrg_mapping.hpp:154-503) ----------------------
    def get_indices(self, cell: int):
        idx = (C.c_uint64 * 3)()
        lvl = C.c_int32()
        check(lib().dccrgx_map_host_indices(C.byref(self._m), C.c_uint64(int(cell)), idx, C.byref(lvl)))
        return tuple(int(v) for v in idx)

    def get_refinement_level(self, cell: int) -> int:
        idx = (C.c_uint64 * 3)()
        lvl = C.c_int32()
        check(lib().dccrgx_map_host_indices(C.byref(self._m), C.c_uint64(int(cell)), idx, C.byref(lvl)))
        return lvl.value

    def get_cell_from_indices(self, idx, lvl: int) -> int:
        a = (C.c_uint64 * 3)(*[int(v) for v in idx])
        out = C.c_uint64()
        check(lib().dccrgx_map_host_cell(C.byref(self._m), a, int(lvl), C.byref(out)))
        return out.value

    def _op(self, op: int, cell: int) -> int:
        out = C.c_uint64()
        check(lib().dccrgx_map_host_op(C.byref(self._m), op, C.c_uint64(int(cell)), C.byref(out)))
        return out.value

    def get_cell_length_in_indices(self, cell: int) -> int:
        return self._op(X.OP_LENGTH_IN_INDICES, cell)

    def get_parent(self, cell: int) -> int:
        return self._op(X.OP_PARENT, cell)

    def get_level_0_parent(self, cell: int) -> int:
        return self._op(X.OP_LEVEL_0_PARENT, cell)

    def get_child(self, cell: int) -> int:
        return self._op(X.OP_CHILD, cell)

    # ---- host arrays (numpy in, numpy out) --------------------------------
    def levels_and_indices(self, cells):
        """(indices (n, 3) uint64 in max-level units, levels int32) of an array of ids."""
        c = np.ascontiguousarray(cells, dtype=np.uint64)
        idx = np.zeros((c.size, 3), dtype=np.uint64)
        lvl = np.zeros(c.size, dtype=np.int32)
        check(lib().dccrgx_map_host_ids_to_indices(C.byref(self._m), c.ctypes.data_as(X._u64p), c.size,
                                                   idx.ctypes.data_as(X._u64p), lvl.ctypes.data_as(X._i32p)))
        return idx, lvl

    def ids_op_host(self, op: int, cells) -> np.ndarray:
        c = np.ascontiguousarray(cells, dtype=np.uint64)
        out = np.zeros(c.size, dtype=np.uint64)
        check(lib().dccrgx_map_host_ids_op(C.byref(self._m), op, c.ctypes.data_as(X._u64p), c.size,
                                           out.ctypes.data_as(X._u64p)))
        return out

    def parents(self, cells) -> np.ndarray:
        return self.ids_op_host(X.OP_PARENT, cells)

    def get_all_children(self, cell: int):
        """dccrg_mapping.hpp:392-442: x fastest, then y, z; error_cell x 8
        for error_cell or a cell at the maximum level.  As in the reference,
        an id beyond the last cell (level -1) is not rejected: its error_index
        corner wraps in unsigned 64-bit arithmetic."""
        lvl = self.get_refinement_level(cell)
        if cell == 0 or lvl >= self.max_ref_lvl:
            return [0] * 8
        i = self.get_indices(cell)
        h = 1 << (self.max_ref_lvl - lvl - 1)
        w = (1 << 64) - 1
        return [self.get_cell_from_indices(((i[0] + dx * h) & w, (i[1] + dy * h) & w, (i[2] + dz * h) & w),
                                           lvl + 1)
                for dz in (0, 1) for dy in (0, 1) for dx in (0, 1)]

    def get_siblings(self, cell: int):
        """dccrg_mapping.hpp:450-471."""
        lvl = self.get_refinement_level(cell)
        if lvl < 0 or lvl > self.max_ref_lvl:
            return [0] * 8
        if lvl == 0:
            return [int(cell)] + [0] * 7
        return self.get_all_children(self.get_parent(cell))

    def ids_to_indices(self, ids, stream: int = 0):
        import torch
        n = ids.numel()
        idx = torch.empty((n, 3), dtype=torch.int64, device=ids.device)
        lvl = torch.empty(n, dtype=torch.int32, device=ids.device)
        check(lib().dccrgx_map_ids_to_indices(C.byref(self._m), ids.data_ptr(), n, idx.data_ptr(),
                                              lvl.data_ptr(), stream or None))
        return idx, lvl

    def indices_to_ids(self, idx, lvl, stream: int = 0):
        import torch
        n = lvl.numel()
        ids = torch.empty(n, dtype=torch.int64, device=lvl.device)
        check(lib().dccrgx_map_indices_to_ids(C.byref(self._m), idx.data_ptr(), lvl.data_ptr(), n,
                                              ids.data_ptr(), stream or None))
        return ids

    def ids_op(self, op: int, ids, stream: int = 0):
        import torch
        out = torch.empty_like(ids)
        check(lib().dccrgx_map_ids_op(C.byref(self._m), op, ids.data_ptr(), ids.numel(),
                                      out.data_ptr(), stream or None))
        return out


class Dccrg:
    """dccrg::Dccrg for the hot path (dccrg.hpp:151-7186)."""

    def __init__(self):
        self._length = (1, 1, 1)
        self._max_ref_lvl = 0
        self._periodic = (False, False, False)
        self._hood_length = 1
        self._h = None
        self.ctx: Optional[Context] = None
        self._fields: Dict[str, Tuple[int, np.dtype]] = {}

    # ---- chained configuration (dccrg.hpp:8242-8361) ---------------------
    def set_initial_length(self, length):
        if any(int(v) == 0 for v in length):
            raise ValueError("all lengths must be > 0 (dccrg.hpp:8244-8254)")
        self._length = tuple(int(v) for v in length)
        return self

    def set_maximum_refinement_level(self, lvl: int):
        self._max_ref_lvl = int(lvl)
        return self

    def set_periodic(self, x: bool, y: bool, z: bool):
        self._periodic = (bool(x), bool(y), bool(z))
        return self

    def set_neighborhood_length(self, n: int):
        self._hood_length = int(n)
        return self

    def set_load_balancing_method(self, method: str):
        # Zoltan stays on the host (north star); the partition is the
        # reference's own non-Zoltan block partition (dccrg.hpp:8098-8145).
        self._lb_method = method
        return self

    def set_initial_partition(self, method: str = "block"):
        """Placement of the level-0 cells at initialize: "block" (contiguous
        ids, dccrg.hpp:8116-8145) or "sfc" (the same per-process counts
        along a Hilbert curve computed on the device; the reference's
        compile-time USE_SFC branch, :8147-8220).  An SFC grid uses the
        explicit layout."""
        m = method.lower()
        if m not in ("block", "sfc"):
            raise ValueError(f"unknown partition {method!r}")
        self._partition = X.PARTITION_SFC if m == "sfc" else X.PARTITION_BLOCK
        return self

    def initialize(self, ctx: Context, leaves: Optional[Sequence[int]] = None):
        """dccrg.hpp:485-562.  leaves: existing cells of a mixed-level grid."""
        self.ctx = ctx
        p = X.GridParams_t()
        p.length = (C.c_uint64 * 3)(*self._length)
        p.max_ref_lvl = self._max_ref_lvl
        p.neighborhood_length = self._hood_length
        p.periodic = (C.c_uint8 * 3)(*[1 if v else 0 for v in self._periodic])
        p.partition = getattr(self, "_partition", X.PARTITION_BLOCK)
        h = C.c_void_p()
        if leaves is None:
            check(lib().dccrgx_grid_create(ctx._h, C.byref(p), None, 0, C.byref(h)))
        else:
            lv = _u64(leaves)
            check(lib().dccrgx_grid_create(ctx._h, C.byref(p), lv.ctypes.data_as(X._u64p), lv.size,
                                           C.byref(h)))
        self._h = h
        info = X.GridInfo_t()
        check(lib().dccrgx_grid_get_info(self._h, C.byref(info)))
        self.info = info
        self.mapping = Mapping(self._length, info.max_ref_lvl)
        return self

    def balance_load(self, use_zoltan: bool = True):
        # without Zoltan the reference's balance_load is a no-op (dccrg.hpp:1048-1062)
        return self

    def close(self):
        if self._h:
            lib().dccrgx_grid_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- adaptive mesh refinement (dccrg.hpp:2456-2806, 3483-3543) ---------
    def _request(self, fn, cell: int) -> bool:
        r = C.c_int32()
        check(fn(self._h, C.c_uint64(int(cell)), C.byref(r)))
        self._refresh_info()  # a uniform grid switches to the explicit layout
        return bool(r.value)

    def refine_completely(self, cell: int) -> bool:
        return self._request(lib().dccrgx_refine_completely, cell)

    def unrefine_completely(self, cell: int) -> bool:
        return self._request(lib().dccrgx_unrefine_completely, cell)

    def dont_unrefine(self, cell: int) -> bool:
        return self._request(lib().dccrgx_dont_unrefine, cell)

    def dont_refine(self, cell: int) -> bool:
        return self._request(lib().dccrgx_dont_refine, cell)

    def request_cells(self, kind: int, ids) -> np.ndarray:
        """The request call `kind` (AMR_REFINE, AMR_DONT_REFINE, AMR_UNREFINE,
        AMR_DONT_UNREFINE) for every id, in order, as one batch (on the device
        for explicit grids); the calls' bool results."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        res = np.zeros(max(ids.size, 1), dtype=np.int32)
        check(lib().dccrgx_amr_request_cells(self._h, kind, ids.ctypes.data_as(X._u64p), ids.size,
                                             res.ctypes.data_as(X._i32p)))
        return res[:ids.size].astype(bool)

    def amr_requests(self):
        """This rank's four pending request sets (refine, dont_refine,
        unrefine, dont_unrefine), for the all-gather of stop_refining."""
        out = []
        for k in range(4):
            n = C.c_size_t()
            check(lib().dccrgx_amr_requests(self._h, k, None, 0, C.byref(n)))
            a = np.zeros(n.value, dtype=np.uint64)
            check(lib().dccrgx_amr_requests(self._h, k, a.ctypes.data_as(X._u64p), a.size, C.byref(n)))
            out.append(a)
        return out

    def stop_refining(self, sorted: bool = True, all_requests=None) -> np.ndarray:
        """Collective (dccrg.hpp:3483-3507).  all_requests: the union over all
        ranks of amr_requests(); gathered with torch.distributed when the
        grid has several ranks and it is not given.  Two phases: every rank
        prepares its new grid, the statuses are all-reduced (torch.distributed),
        and all ranks adopt or all keep the old grid with the requests pending
        -- a failure on any rank raises on every rank.  With several ranks and
        no torch.distributed the agreement is impossible and this raises:
        ranks held in one process go through stop_refining_all, which runs
        the two phases across them."""
        multi = self.ctx.comm_size > 1
        if multi and not _dist_ready():
            raise X.DccrgxError(X.DCCRGX_ESTATE, "stop_refining with several ranks needs torch.distributed for the "
                                                 "ranks' status agreement (ranks in one process: stop_refining_all)")
        if multi and all_requests is None:
            import torch.distributed as dist
            mine = self.amr_requests()
            got = [None] * self.ctx.comm_size
            dist.all_gather_object(got, [a.tolist() for a in mine])
            all_requests = [np.unique(np.concatenate([np.asarray(g[k], dtype=np.uint64) for g in got]))
                            for k in range(4)]
        st, err = self.stop_refining_prepare(all_requests)
        ok = st == X.DCCRGX_OK
        all_ok = ok
        if multi:
            import torch
            import torch.distributed as dist
            t = torch.tensor([1 if ok else 0], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            all_ok = bool(t.item())
        self.stop_refining_finish(all_ok)
        if not ok:
            raise X.DccrgxError(st, err)
        if not all_ok:
            raise X.DccrgxError(X.DCCRGX_ESTATE, "stop_refining failed on another rank; requests stay pending")
        return self.get_new_cells()

    def stop_refining_count(self) -> int:
        """stop_refining of a one-rank grid from its own requests, returning
        the number of new cells instead of the list (get_new_cells has it)."""
        if self.ctx.comm_size != 1:
            raise X.DccrgxError(X.DCCRGX_ESTATE, "stop_refining_count is the one-rank form")
        n_new = C.c_size_t()
        check(lib().dccrgx_stop_refining(self._h, None, None, C.byref(n_new)))
        self._refresh_info()
        return int(n_new.value)

    def stop_refining_prepare(self, all_requests=None):
        """Phase one (dccrgx_stop_refining_prepare): (status, error message);
        the grid stays the old one until stop_refining_finish."""
        n_new = C.c_size_t()
        if all_requests is None:  # this rank's own requests (they stay on the device)
            st = lib().dccrgx_stop_refining_prepare(self._h, None, None, C.byref(n_new))
        else:
            sets = [_u64(a) for a in all_requests]
            ptrs = (X._u64p * 4)(*[a.ctypes.data_as(X._u64p) for a in sets])
            counts = (C.c_size_t * 4)(*[a.size for a in sets])
            st = lib().dccrgx_stop_refining_prepare(self._h, ptrs, counts, C.byref(n_new))
        err = lib().dccrgx_last_error().decode(errors="replace") if st != X.DCCRGX_OK else ""
        return st, err

    def stop_refining_finish(self, commit: bool):
        """Phase two: adopt the prepared grid (commit) or drop it."""
        check(lib().dccrgx_stop_refining_finish(self._h, 1 if commit else 0))
        self._refresh_info()
        return self

    def get_new_cells(self) -> np.ndarray:
        return self._id_list(lib().dccrgx_get_new_cells)

    def get_removed_cells(self, sorted: bool = True) -> np.ndarray:
        return self._id_list(lib().dccrgx_get_removed_cells)

    def clear_refined_unrefined_data(self):
        check(lib().dccrgx_clear_refined_unrefined_data(self._h))
        return self

    def _id_list(self, fn) -> np.ndarray:
        n = C.c_size_t()
        check(fn(self._h, None, 0, C.byref(n)))
        out = np.zeros(n.value, dtype=np.uint64)
        check(fn(self._h, out.ctypes.data_as(X._u64p), out.size, C.byref(n)))
        return out

    def _refresh_info(self):
        info = X.GridInfo_t()
        check(lib().dccrgx_grid_get_info(self._h, C.byref(info)))
        self.info = info

    # ---- queries ------------------------------------------------------------
    def get_rank(self) -> int:
        return self.ctx.rank

    def get_comm_size(self) -> int:
        return self.ctx.comm_size

    def get_maximum_refinement_level(self) -> int:
        return self.info.max_ref_lvl

    @property
    def n_local(self) -> int:
        return self.info.n_local

    def _cells(self, which: int, hood: int) -> np.ndarray:
        n = C.c_size_t()
        st = lib().dccrgx_get_cells(self._h, hood, which, None, 0, C.byref(n))
        if st not in (X.DCCRGX_OK, 5):
            check(st)
        out = np.zeros(n.value, dtype=np.uint64)
        check(lib().dccrgx_get_cells(self._h, hood, which, out.ctypes.data_as(X._u64p), n.value,
                                     C.byref(n)))
        return out

    def local_cells(self, hood: int = DEFAULT_NEIGHBORHOOD_ID) -> np.ndarray:
        return self._cells(X.CELLS_LOCAL, hood)

    def inner_cells(self, hood: int = DEFAULT_NEIGHBORHOOD_ID) -> np.ndarray:
        return self._cells(X.CELLS_INNER, hood)

    def outer_cells(self, hood: int = DEFAULT_NEIGHBORHOOD_ID) -> np.ndarray:
        return self._cells(X.CELLS_OUTER, hood)

    def remote_cells(self, hood: int = DEFAULT_NEIGHBORHOOD_ID) -> np.ndarray:
        return self._cells(X.CELLS_REMOTE, hood)

    def get_all_cells(self) -> np.ndarray:
        """Every leaf of the grid, ascending (Dccrg::get_all_cells, dccrg.hpp:3557-3590)."""
        n = C.c_size_t()
        s = lib().dccrgx_get_all_cells(self._h, None, 0, C.byref(n))
        if s not in (X.DCCRGX_OK, 5):  # 5: ERANGE, the sizing call
            check(s)
        out = np.zeros(n.value, dtype=np.uint64)
        if n.value:
            check(lib().dccrgx_get_all_cells(self._h, out.ctypes.data_as(X._u64p), out.size, C.byref(n)))
        return out

    def neighbor_list_stats(self, hood: int = DEFAULT_NEIGHBORHOOD_ID) -> dict:
        """The device lists this rank holds (dccrgx_neighbor_list_stats)."""
        out = (C.c_uint64 * 4)()
        check(lib().dccrgx_neighbor_list_stats(self._h, hood, out))
        return {"rows": int(out[0]), "nof_entries": int(out[1]), "nto_entries": int(out[2]), "bytes": int(out[3])}

    def stencil_view(self, hood: int = DEFAULT_NEIGHBORHOOD_ID, region: int = X.REGION_ALL) -> "X.StencilView_t":
        """The device data a user stencil walks (dccrgx_stencil_view_get; the
        C++ side is include/dccrgx_stencil.hpp's for_each_cell): the region's
        cell count, and for each cell its neighbors_of in the iteration cache's
        order (dccrg.hpp:11590-11640)."""
        v = X.StencilView_t()
        check(lib().dccrgx_stencil_view_get(self._h, hood, region, C.byref(v)))
        return v

    def neighbors_of(self, cells: np.ndarray, hood: int = DEFAULT_NEIGHBORHOOD_ID):
        """Batched get_neighbors_of: (row_ptr, ids, offsets[x,y,z]) as numpy."""
        import torch
        dev = torch.device("cuda", self.ctx.device)
        c = torch.from_numpy(_u64(cells).view(np.int64)).to(dev)
        n = c.numel()
        with _OnLibraryStream(self.ctx, dev):
            row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            check(lib().dccrgx_neighbors_of(self._h, hood, c.data_ptr(), n, row.data_ptr(), None, None, 0, None))
            total = int(row[-1].item())
            ids = torch.zeros(max(total, 1), dtype=torch.int64, device=dev)
            off = torch.zeros((max(total, 1), 3), dtype=torch.int32, device=dev)
            check(lib().dccrgx_neighbors_of(self._h, hood, c.data_ptr(), n, row.data_ptr(), ids.data_ptr(),
                                            off.data_ptr(), total, None))
            return (row.cpu().numpy().astype(np.uint64), ids[:total].cpu().numpy().view(np.uint64),
                    off[:total].cpu().numpy())

    def gather_neighbors(self, name: str, cells=None, hood: int = DEFAULT_NEIGHBORHOOD_ID):
        """Neighbor gather for user stencils (dccrgx_gather_neighbors): for
        local cells (default: all, ascending), torch tensors (row_ptr,
        values) with values[row[i]:row[i+1]] = the field element of each
        get_neighbors_of(cells[i]) entry, in list order (ghosts from their
        copies)."""
        import torch
        dev = torch.device("cuda", self.ctx.device)
        fid, dt = self._fields[name]
        c = self.local_cells() if cells is None else cells
        ct = torch.from_numpy(_u64(c).view(np.int64)).to(dev)
        n = ct.numel()
        with _OnLibraryStream(self.ctx, dev) as ls:
            row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            check(lib().dccrgx_gather_neighbors(self._h, hood, fid, ct.data_ptr(), n, row.data_ptr(), None, 0, None))
            total = int(row[-1].item())
            out = torch.zeros(max(total, 1) * dt.itemsize, dtype=torch.uint8, device=dev)
            check(lib().dccrgx_gather_neighbors(self._h, hood, fid, ct.data_ptr(), n, row.data_ptr(),
                                                out.data_ptr(), out.numel(), None))
            ls.hand_over(row, out)
        return row, out[:total * dt.itemsize]

    def neighbors_to(self, cells: np.ndarray, hood: int = DEFAULT_NEIGHBORHOOD_ID):
        import torch
        dev = torch.device("cuda", self.ctx.device)
        c = torch.from_numpy(_u64(cells).view(np.int64)).to(dev)
        n = c.numel()
        with _OnLibraryStream(self.ctx, dev):
            row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            check(lib().dccrgx_neighbors_to(self._h, hood, c.data_ptr(), n, row.data_ptr(), None, 0, None))
            total = int(row[-1].item())
            ids = torch.zeros(max(total, 1), dtype=torch.int64, device=dev)
            check(lib().dccrgx_neighbors_to(self._h, hood, c.data_ptr(), n, row.data_ptr(), ids.data_ptr(),
                                            total, None))
            return row.cpu().numpy().astype(np.uint64), ids[:total].cpu().numpy().view(np.uint64)

    def get_neighbors_of(self, cell: int, hood: int = DEFAULT_NEIGHBORHOOD_ID):
        """dccrg.hpp:836-883 for one cell: [(id, (x, y, z)), ...] in reference order."""
        row, ids, off = self.neighbors_of(np.array([cell]), hood)
        return [(int(i), tuple(int(v) for v in o)) for i, o in zip(ids, off)]

    def face_neighbors_of(self, cells: np.ndarray):
        """Batched get_face_neighbors_of (dccrg.hpp:2828-2955) on the device:
        (row_ptr, ids, dirs) as numpy."""
        import torch
        dev = torch.device("cuda", self.ctx.device)
        c = torch.from_numpy(_u64(cells).view(np.int64)).to(dev)
        n = c.numel()
        with _OnLibraryStream(self.ctx, dev):
            row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            cap = 24 * max(n, 1)
            ids = torch.zeros(cap, dtype=torch.int64, device=dev)
            dirs = torch.zeros(cap, dtype=torch.int32, device=dev)
            check(lib().dccrgx_face_neighbors_of(self._h, c.data_ptr(), n, row.data_ptr(), ids.data_ptr(),
                                                 dirs.data_ptr(), cap, None))
            total = int(row[-1].item())
            return (row.cpu().numpy().astype(np.uint64), ids[:total].cpu().numpy().view(np.uint64),
                    dirs[:total].cpu().numpy())

    def get_face_neighbors_of(self, cell: int):
        """dccrg.hpp:2828-2955 for one cell: [(id, direction), ...]."""
        _, ids, dirs = self.face_neighbors_of(np.array([cell]))
        return [(int(i), int(d)) for i, d in zip(ids, dirs)]

    def get_neighbors_to(self, cell: int, hood: int = DEFAULT_NEIGHBORHOOD_ID):
        row, ids = self.neighbors_to(np.array([cell]), hood)
        return [int(i) for i in ids]

    def add_neighborhood(self, hood_id: int, items) -> bool:
        """dccrg.hpp:6491-6663: False where the reference returns false."""
        it = np.ascontiguousarray(items, dtype=np.int32).reshape(-1, 3)
        st = lib().dccrgx_add_neighborhood(self._h, hood_id, it.ctypes.data_as(X._i32p), len(it))
        if st == 1:  # EINVAL
            return False
        check(st)
        return True

    def remove_neighborhood(self, hood_id: int):
        check(lib().dccrgx_remove_neighborhood(self._h, hood_id))
        return self

    def _peer_lists(self, send: int, hood: int) -> Dict[int, List[int]]:
        n = C.c_size_t()
        st = lib().dccrgx_get_peers(self._h, hood, send, None, None, 0, C.byref(n))
        if st not in (X.DCCRGX_OK, 5):
            check(st)
        peers = np.zeros(n.value, dtype=np.int32)
        counts = np.zeros(n.value, dtype=np.uint64)
        check(lib().dccrgx_get_peers(self._h, hood, send, peers.ctypes.data_as(X._i32p),
                                     counts.ctypes.data_as(X._u64p), n.value, C.byref(n)))
        out = {}
        for p, k in zip(peers, counts):
            ids = np.zeros(int(k), dtype=np.uint64)
            m = C.c_size_t()
            check(lib().dccrgx_get_peer_cells(self._h, hood, send, int(p), ids.ctypes.data_as(X._u64p),
                                              int(k), C.byref(m)))
            out[int(p)] = ids.tolist()
        return out

    def _update_cells(self, send: int, hood: int) -> int:
        n = C.c_size_t()
        st = lib().dccrgx_get_peers(self._h, hood, send, None, None, 0, C.byref(n))
        if st == 7:  # DCCRGX_ENOTFOUND: dccrg.hpp:5454-5456
            return (1 << 64) - 1
        if st not in (X.DCCRGX_OK, 5):
            check(st)
        counts = np.zeros(n.value, dtype=np.uint64)
        check(lib().dccrgx_get_peers(self._h, hood, send, None, counts.ctypes.data_as(X._u64p), n.value,
                                     C.byref(n)))
        return int(counts.sum())

    def get_number_of_update_send_cells(self, hood: int = DEFAULT_NEIGHBORHOOD_ID) -> int:
        """dccrg.hpp:5428-5480: cells sent per update (a cell sent to N
        processes counts N times); maximum uint64 for an unknown id."""
        return self._update_cells(1, hood)

    def get_number_of_update_receive_cells(self, hood: int = DEFAULT_NEIGHBORHOOD_ID) -> int:
        """dccrg.hpp:5489-5536."""
        return self._update_cells(0, hood)

    def get_cells_to_send(self, hood: int = DEFAULT_NEIGHBORHOOD_ID) -> Dict[int, List[int]]:
        """dccrg.hpp:7008-7020: per receiving process, ascending cell ids."""
        return self._peer_lists(1, hood)

    def get_cells_to_receive(self, hood: int = DEFAULT_NEIGHBORHOOD_ID) -> Dict[int, List[int]]:
        return self._peer_lists(0, hood)

    # ---- cell data ------------------------------------------------------------
    def add_field(self, name: str, dtype=np.uint32) -> int:
        dt = np.dtype(dtype)
        fid = C.c_int32()
        check(lib().dccrgx_field_create(self._h, dt.itemsize, C.byref(fid)))
        self._fields[name] = (fid.value, dt)
        return fid.value

    def add_variable_field(self, name: str, dtype=np.int32) -> int:
        """A field with a per-cell number of elements (tests/variable_data_size)."""
        dt = np.dtype(dtype)
        fid = C.c_int32()
        check(lib().dccrgx_field_create_variable(self._h, dt.itemsize, C.byref(fid)))
        self._fields[name] = (fid.value, dt)
        return fid.value

    def resize(self, name: str, cells, counts):
        """Element counts of local cells or ghosts (std::vector::resize)."""
        fid, _ = self._fields[name]
        c = _u64(cells)
        n = np.ascontiguousarray(np.broadcast_to(np.asarray(counts, dtype=np.uint32), c.shape))
        check(lib().dccrgx_field_resize(self._h, fid, c.ctypes.data_as(X._u64p),
                                        n.ctypes.data_as(C.POINTER(C.c_uint32)), c.size))

    def get_counts(self, name: str, cells) -> np.ndarray:
        fid, _ = self._fields[name]
        c = _u64(cells)
        out = np.zeros(c.size, dtype=np.uint32)
        check(lib().dccrgx_field_get_counts(self._h, fid, c.ctypes.data_as(X._u64p), c.size,
                                            out.ctypes.data_as(C.POINTER(C.c_uint32))))
        return out

    def write_cells(self, name: str, cells, values):
        """values: one array per cell, or the cells' elements concatenated."""
        fid, dt = self._fields[name]
        c = _u64(cells)
        if isinstance(values, (list, tuple)):
            values = np.concatenate([np.asarray(v, dtype=dt).ravel() for v in values]) if values else \
                np.zeros(0, dtype=dt)
        v = np.ascontiguousarray(values, dtype=dt)
        check(lib().dccrgx_field_write_cells(self._h, fid, c.ctypes.data_as(X._u64p), c.size, v.ctypes.data,
                                             v.nbytes))

    def read_cells(self, name: str, cells):
        """One array per cell (operator[] on local cells and ghosts)."""
        fid, dt = self._fields[name]
        c = _u64(cells)
        nbytes = C.c_size_t()
        check(lib().dccrgx_field_read_cells(self._h, fid, c.ctypes.data_as(X._u64p), c.size, None, 0,
                                            C.byref(nbytes)))
        buf = np.zeros(nbytes.value // dt.itemsize, dtype=dt)
        check(lib().dccrgx_field_read_cells(self._h, fid, c.ctypes.data_as(X._u64p), c.size, buf.ctypes.data,
                                            buf.nbytes, C.byref(nbytes)))
        counts = self.get_counts(name, c)
        return np.split(buf, np.cumsum(counts)[:-1]) if c.size else []

    def field_id(self, name: str) -> int:
        return self._fields[name][0]

    def checksum(self, name: str) -> Tuple[int, int]:
        """(sum of values, sum of value * splitmix64(id)) mod 2^64 of a 4-byte
        field over the local cells, on the device (dccrgx_field_checksum)."""
        out = (C.c_uint64 * 2)()
        check(lib().dccrgx_field_checksum(self._h, self.field_id(name), out))
        return int(out[0]), int(out[1])

    def write_local(self, name: str, values: np.ndarray):
        """values: one element per local cell, ascending ids; a field whose
        element is an array (e.g. np.dtype((np.uint64, 9))) takes (n, ...)."""
        fid, dt = self._fields[name]
        base, shape = (dt.base, dt.shape) if dt.subdtype is not None else (dt, ())
        v = np.ascontiguousarray(values, dtype=base).reshape((-1,) + shape)
        check(lib().dccrgx_field_write_local(self._h, fid, v.ctypes.data, v.shape[0]))

    def read_local(self, name: str) -> np.ndarray:
        fid, dt = self._fields[name]
        base, shape = (dt.base, dt.shape) if dt.subdtype is not None else (dt, ())
        out = np.zeros((self.info.n_local,) + shape, dtype=base)
        check(lib().dccrgx_field_read_local(self._h, fid, out.ctypes.data, self.info.n_local))
        return out

    def read_remote(self, name: str, hood: int = DEFAULT_NEIGHBORHOOD_ID) -> np.ndarray:
        fid, dt = self._fields[name]
        n = len(self.remote_cells(hood))
        base, shape = (dt.base, dt.shape) if dt.subdtype is not None else (dt, ())
        out = np.zeros((n,) + shape, dtype=base)
        check(lib().dccrgx_field_read_remote(self._h, hood, fid, out.ctypes.data, n))
        return out

    def _fids(self, names) -> np.ndarray:
        if names is None:
            names = list(self._fields)
        return np.array([self._fields[n][0] for n in names], dtype=np.int32)

    # ---- grid data files (dccrg.hpp:1109-2427) -------------------------------
    def save_sizes(self, fields) -> Tuple[int, int]:
        """This rank's (cells, data bytes) for a save of `fields`."""
        f = self._fids(fields)
        n, b = C.c_uint64(), C.c_uint64()
        check(lib().dccrgx_save_sizes(self._h, f.ctypes.data_as(X._i32p), f.size, C.byref(n), C.byref(b)))
        return n.value, b.value

    def save_grid_data(self, name: str, offset: int = 0, header: bytes = b"", fields=None,
                       geometry: Optional[bytes] = None, all_sizes=None) -> bool:
        """Dccrg::save_grid_data (dccrg.hpp:1109-1712).  A cell's data is
        `fields` in order (the members its get_mpi_datatype() would list).
        geometry: the stored geometry blob (no_geometry() by default).
        all_sizes: every rank's save_sizes() in rank order; all-gathered with
        torch.distributed when the grid has several ranks and it is not given."""
        f = self._fids(fields)
        geometry = no_geometry() if geometry is None else bytes(geometry)
        mine = self.save_sizes(fields)
        if all_sizes is None:
            if self.ctx.comm_size == 1:
                all_sizes = [mine]
            else:
                import torch.distributed as dist
                all_sizes = [None] * self.ctx.comm_size
                dist.all_gather_object(all_sizes, mine)
        r = self.ctx.rank
        assert tuple(all_sizes[r]) == tuple(mine), "all_sizes does not match this rank's share"
        total = sum(int(n) for n, _ in all_sizes)
        cb = sum(int(n) for n, _ in all_sizes[:r])
        bb = sum(int(b) for _, b in all_sizes[:r])
        hb = bytes(header)
        check(lib().dccrgx_save_grid_data(self._h, name.encode(), offset, hb, len(hb), geometry, len(geometry),
                                          total, cb, bb, f.ctypes.data_as(X._i32p), f.size))
        return True

    @staticmethod
    def read_file_info(name: str, offset: int = 0, header_bytes: int = 0):
        """(file info, header bytes, geometry blob) of a grid data file."""
        info = X.FileInfo_t()
        hdr = C.create_string_buffer(max(header_bytes, 1))
        check(lib().dccrgx_file_read_info(name.encode(), offset, hdr, header_bytes, C.byref(info), None, 0))
        geo = C.create_string_buffer(int(info.geometry_bytes))
        check(lib().dccrgx_file_read_info(name.encode(), offset, hdr, header_bytes, C.byref(info), geo,
                                          info.geometry_bytes))
        return info, hdr.raw[:header_bytes], geo.raw

    @classmethod
    def start_loading_grid_data(cls, ctx: "Context", name: str, offset: int = 0, header_bytes: int = 0,
                                partition: str = "block"):
        """Dccrg::start_loading_grid_data (dccrg.hpp:1815-2105): a grid of the
        file's cells on `ctx`, placed by `partition` ("block" or "sfc", as
        set_initial_partition; the file records no placement).  Returns
        (grid, header bytes, geometry blob); add fields, then
        continue_loading_grid_data(fields), then finish_loading_grid_data()."""
        info, hdr, geo = cls.read_file_info(name, offset, header_bytes)
        g = cls()
        p = info.params
        if partition.lower() not in ("block", "sfc"):
            raise ValueError(f"unknown partition {partition!r}")
        p.partition = X.PARTITION_SFC if partition.lower() == "sfc" else X.PARTITION_BLOCK
        g._partition = p.partition
        g._length = tuple(int(v) for v in p.length)
        g._max_ref_lvl = int(p.max_ref_lvl)
        g._periodic = tuple(bool(v) for v in p.periodic)
        g._hood_length = int(p.neighborhood_length)
        g.ctx = ctx
        h = C.c_void_p()
        check(lib().dccrgx_grid_load(ctx._h, name.encode(), C.byref(info), C.byref(h)))
        g._h = h
        g._refresh_info()
        g.mapping = Mapping(g._length, g.info.max_ref_lvl)
        return g, hdr, geo

    def continue_loading_grid_data(self, fields):
        """dccrg.hpp:2134-2390: the next bytes of every local cell's record
        into `fields` (variable fields sized beforehand)."""
        f = self._fids(fields)
        check(lib().dccrgx_load_cell_data(self._h, f.ctypes.data_as(X._i32p), f.size))
        return True

    def finish_loading_grid_data(self):
        check(lib().dccrgx_finish_loading_grid_data(self._h))
        return True

    # ---- halo (dccrg.hpp:978-1014, 5046-5413) --------------------------------
    def update_copies_of_remote_neighbors(self, hood: int = DEFAULT_NEIGHBORHOOD_ID, fields=None):
        f = self._fids(fields)
        # no device-wide wait: the ghosts' writes are queued on the library's
        # compute stream (dccrgx_halo_wait orders it after the exchange), where
        # every later read of the fields runs
        check(lib().dccrgx_halo_update(self._h, hood, f.ctypes.data_as(X._i32p), f.size))
        # quirk kept: with the default id the reference returns false (dccrg.hpp:1001-1003)
        return hood != DEFAULT_NEIGHBORHOOD_ID

    def start_remote_neighbor_copy_updates(self, hood: int = DEFAULT_NEIGHBORHOOD_ID, fields=None):
        f = self._fids(fields)
        check(lib().dccrgx_halo_start(self._h, hood, f.ctypes.data_as(X._i32p), f.size))
        return True

    def wait_remote_neighbor_copy_updates(self, hood: int = DEFAULT_NEIGHBORHOOD_ID):
        check(lib().dccrgx_halo_wait(self._h, hood, X.WAIT_ALL))
        return True

    def wait_remote_neighbor_copy_update_receives(self, hood: int = DEFAULT_NEIGHBORHOOD_ID):
        check(lib().dccrgx_halo_wait(self._h, hood, X.WAIT_RECEIVES))
        return True

    def wait_remote_neighbor_copy_update_sends(self, hood: int = DEFAULT_NEIGHBORHOOD_ID):
        check(lib().dccrgx_halo_wait(self._h, hood, X.WAIT_SENDS))
        return True

    def pack_to(self, peer: int, dst_ptr: int, cap: int, hood: int = DEFAULT_NEIGHBORHOOD_ID,
                fields=None) -> int:
        f = self._fids(fields)
        n = C.c_size_t()
        check(lib().dccrgx_halo_pack_to(self._h, hood, f.ctypes.data_as(X._i32p), f.size, peer, dst_ptr,
                                        cap, C.byref(n)))
        return n.value

    def unpack_from(self, peer: int, src_ptr: int, nbytes: int, hood: int = DEFAULT_NEIGHBORHOOD_ID,
                    fields=None):
        f = self._fids(fields)
        check(lib().dccrgx_halo_unpack_from(self._h, hood, f.ctypes.data_as(X._i32p), f.size, peer,
                                            src_ptr, nbytes))

    def halo_self(self, hood: int = DEFAULT_NEIGHBORHOOD_ID, fields=None):
        f = self._fids(fields)
        check(lib().dccrgx_halo_self(self._h, hood, f.ctypes.data_as(X._i32p), f.size))

    # ---- game of life stencil ----------------------------------------------
    def gol_compute(self, fin: str, fout: str, fcnt: str, region: int = X.REGION_ALL,
                    hood: int = DEFAULT_NEIGHBORHOOD_ID):
        check(lib().dccrgx_gol_compute(self._h, hood, self.field_id(fin), self.field_id(fout),
                                       self.field_id(fcnt), region))

    def gol_step(self, fin: str, fout: str, fcnt: str, hood: int = DEFAULT_NEIGHBORHOOD_ID):
        check(lib().dccrgx_gol_step(self._h, hood, self.field_id(fin), self.field_id(fout),
                                    self.field_id(fcnt)))

    def gol_amr_step(self, field: str, hood: int = DEFAULT_NEIGHBORHOOD_ID):
        """tests/game_of_life/solve.hpp:40-170 get_live_neighbors on a 9 x u64
        field (cell.hpp:47): record, halo, spread + apply."""
        check(lib().dccrgx_gol_amr_step(self._h, hood, self.field_id(field)))

    def gol_amr_phase(self, field: str, phase: int, hood: int = DEFAULT_NEIGHBORHOOD_ID):
        """One phase of gol_amr_step (X.GOLH_RECORD / X.GOLH_SPREAD_APPLY)."""
        check(lib().dccrgx_gol_amr_phase(self._h, hood, self.field_id(field), phase))

    # ---- advection, tests/advection/solve.hpp ------------------------------
    ADVECT_FIELDS = ("density", "flux", "vx", "vy", "vz", "length_x", "length_y", "length_z")

    def _advect_fields(self, names=None):
        """names: mapping from the Cell::data members (cell.hpp:34-44) to
        field names; default: fields named after the members (made once: a
        field keeps its id)."""
        if not names:
            f = getattr(self, "_adv_default", None)
            if f is None:
                f = self._adv_default = X.AdvectFields_t(*[self.field_id(m) for m in self.ADVECT_FIELDS])
            return f
        return X.AdvectFields_t(*[self.field_id(names.get(m, m)) for m in self.ADVECT_FIELDS])

    def add_advection_fields(self):
        for m in self.ADVECT_FIELDS:
            self.add_field(m, np.float64)

    def calculate_fluxes(self, dt: float, solve_inner: bool, hood: int = DEFAULT_NEIGHBORHOOD_ID,
                         names=None, region=None):
        """solve.hpp:44-247: inner cells (solve_inner) or outer cells."""
        f = self._advect_fields(names)
        if region is None:
            region = X.REGION_INNER if solve_inner else X.REGION_OUTER
        check(lib().dccrgx_advect_fluxes(self._h, hood, C.byref(f), dt, region))

    def apply_fluxes(self, names=None):
        f = self._advect_fields(names)
        check(lib().dccrgx_advect_apply(self._h, C.byref(f)))

    def max_time_step(self, names=None) -> float:
        """Local part of solve.hpp:302-332 (reduce with MIN across ranks)."""
        f = self._advect_fields(names)
        out = C.c_double()
        check(lib().dccrgx_advect_max_time_step(self._h, C.byref(f), C.byref(out)))
        return out.value

    def advect_step(self, dt: float, hood: int = DEFAULT_NEIGHBORHOOD_ID, names=None):
        f = self._advect_fields(names)
        s = lib().dccrgx_advect_step(self._h, hood, f, dt)
        if s:
            check(s)

    def kernel_timer(self, reset: int = 0):
        ms = C.c_double()
        n = C.c_uint64()
        check(lib().dccrgx_kernel_timer(self._h, reset, C.byref(ms), C.byref(n)))
        return ms.value, n.value
