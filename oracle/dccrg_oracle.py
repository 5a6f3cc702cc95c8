"""TEST INFRASTRUCTURE ONLY -- Python face of the CPU oracle.

ctypes wrapper over ``oracle/_build/libdccrg_oracle.so`` (the plain-C
restatement in ``dccrg_oracle.c``) plus pure-Python restatements of the
reference's per-rank bookkeeping, each citing the reference file:line it
follows.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker (or the
timed CPU baseline).  The product package ``dccrg_amd`` never imports it.

Parity pinning: see ``oracle/dccrg_oracle.h`` -- the reference is unbuildable
in this image (it needs Boost.TTI / Zoltan headers the image lacks), so this
restatement is pinned by the reference tests' own known answers
(``tests/golden/*.json``) and the survey's recorded reference outputs.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Dict, List, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libdccrg_oracle.so")

ERROR_CELL = 0
ERROR_INDEX = 0xFFFFFFFFFFFFFFFF
DEFAULT_NEIGHBORHOOD_ID = -0xDCC  # dccrg.hpp:99


def build() -> str:
    """Compile the C restatement (gcc) into oracle/_build/."""
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        u64p = C.POINTER(C.c_uint64)
        i32p = C.POINTER(C.c_int32)
        u32p = C.POINTER(C.c_uint32)
        L.dox_mapping_init.argtypes = [C.c_void_p, u64p, C.c_int32]
        L.dox_max_possible_refinement_level.argtypes = [u64p]
        L.dox_get_cell_from_indices.restype = C.c_uint64
        L.dox_get_cell_from_indices.argtypes = [C.c_void_p, u64p, C.c_int]
        L.dox_get_indices.argtypes = [C.c_void_p, C.c_uint64, u64p]
        L.dox_get_refinement_level.argtypes = [C.c_void_p, C.c_uint64]
        for f in ("dox_get_cell_length_in_indices", "dox_get_parent", "dox_get_child",
                  "dox_get_level_0_parent"):
            getattr(L, f).restype = C.c_uint64
            getattr(L, f).argtypes = [C.c_void_p, C.c_uint64]
        L.dox_get_all_children.argtypes = [C.c_void_p, C.c_uint64, u64p]
        L.dox_get_siblings.argtypes = [C.c_void_p, C.c_uint64, u64p]
        L.dox_map_ids_to_indices.argtypes = [C.c_void_p, u64p, C.c_size_t, u64p, i32p]
        L.dox_map_indices_to_ids.argtypes = [C.c_void_p, u64p, i32p, C.c_size_t, u64p]
        L.dox_default_neighborhood.restype = C.c_size_t
        L.dox_default_neighborhood.argtypes = [C.c_uint, i32p]
        L.dox_block_first_cell.restype = C.c_uint64
        L.dox_block_first_cell.argtypes = [C.c_uint64] * 3
        L.dox_block_owner.restype = C.c_uint64
        L.dox_block_owner.argtypes = [C.c_uint64] * 3
        L.dox_grid_create.restype = C.c_void_p
        L.dox_grid_create.argtypes = [u64p, C.c_int32, C.POINTER(C.c_uint8), u64p, C.c_size_t]
        L.dox_grid_destroy.argtypes = [C.c_void_p]
        L.dox_grid_exists.argtypes = [C.c_void_p, C.c_uint64]
        L.dox_grid_size.restype = C.c_size_t
        L.dox_grid_size.argtypes = [C.c_void_p]
        L.dox_grid_cells.restype = C.c_size_t
        L.dox_grid_cells.argtypes = [C.c_void_p, u64p, C.c_size_t]
        L.dox_get_existing_cell.restype = C.c_uint64
        L.dox_get_existing_cell.argtypes = [C.c_void_p, u64p, C.c_int, C.c_int]
        L.dox_grid_get_child.restype = C.c_uint64
        L.dox_grid_get_child.argtypes = [C.c_void_p, C.c_uint64]
        L.dox_update_neighbors_.argtypes = [C.c_void_p, C.c_uint64, u64p]
        L.dox_find_neighbors_of.restype = C.c_long
        L.dox_find_neighbors_of.argtypes = [C.c_void_p, C.c_uint64, i32p, C.c_size_t, u64p, i32p,
                                            C.c_size_t]
        L.dox_find_neighbors_to.restype = C.c_long
        L.dox_find_neighbors_to.argtypes = [C.c_void_p, C.c_uint64, i32p, C.c_size_t, u64p,
                                            C.c_size_t]
        L.dox_get_face_neighbors_of.restype = C.c_long
        L.dox_get_face_neighbors_of.argtypes = [C.c_void_p, C.c_uint64, u64p, i32p, C.c_size_t]
        L.dox_gol_count.argtypes = [C.c_size_t, u64p, u32p, u32p, u32p]
        L.dox_gol_apply.argtypes = [C.c_size_t, u32p, u32p]
        L.dox_num_threads.restype = C.c_int
        L.dox_set_num_threads.argtypes = [C.c_int]
        L.dox_build_uniform_slot_lists.restype = C.c_long
        L.dox_build_uniform_slot_lists.argtypes = [C.c_void_p, C.c_uint, u64p, u32p, C.c_size_t]
        f64p = C.POINTER(C.c_double)
        L.dox_advect_fluxes.restype = C.c_long
        L.dox_advect_fluxes.argtypes = [C.c_size_t, u32p, u64p, u32p, i32p, C.POINTER(C.c_uint8), u64p] + \
            [f64p] * 8 + [C.c_double]
        L.dox_advect_apply.argtypes = [C.c_size_t, u32p, f64p, f64p]
        L.dox_advect_max_time_step.restype = C.c_double
        L.dox_advect_max_time_step.argtypes = [C.c_size_t, u32p] + [f64p] * 6
        L.dox_poisson_solve.restype = C.c_long
        L.dox_poisson_solve.argtypes = [C.c_size_t, u32p, C.c_int, C.POINTER(C.c_size_t), u64p, u32p, i32p] + \
            [f64p] * 11 + [C.c_uint, C.c_uint, C.c_double, C.c_double, C.c_double, f64p]
        _lib = L
    return _lib


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(C.POINTER(t))


class _MappingStruct(C.Structure):
    _fields_ = [("length", C.c_uint64 * 3), ("max_ref_lvl", C.c_int32), ("pad_", C.c_int32),
                ("last_cell", C.c_uint64)]


def default_neighborhood(hood_length: int) -> np.ndarray:
    """dccrg.hpp:8017-8076 -- the default neighborhood_of items, shape (K, 3)."""
    out = np.zeros((343, 3), dtype=np.int32)
    n = lib().dox_default_neighborhood(hood_length, _p(out, C.c_int32))
    return out[:n].copy()


def neighborhood_to(items: np.ndarray) -> np.ndarray:
    """dccrg.hpp:8070-8075: hood_to = -hood_of."""
    return (-np.asarray(items, dtype=np.int32)).copy()


class Mapping:
    """dccrg_mapping.hpp:55-690 restated (scalar + batched)."""

    def __init__(self, length: Sequence[int], max_ref_lvl: int = 0):
        self._m = _MappingStruct()
        ln = np.array(length, dtype=np.uint64)
        if lib().dox_mapping_init(C.byref(self._m), _p(ln, C.c_uint64), int(max_ref_lvl)) != 0:
            raise ValueError("invalid mapping parameters")

    @property
    def max_ref_lvl(self) -> int:
        return self._m.max_ref_lvl

    @property
    def last_cell(self) -> int:
        return self._m.last_cell

    @property
    def length(self):
        return tuple(self._m.length)

    def get_cell_from_indices(self, idx, lvl: int) -> int:
        a = np.array(idx, dtype=np.uint64)
        return lib().dox_get_cell_from_indices(C.byref(self._m), _p(a, C.c_uint64), int(lvl))

    def get_indices(self, cell: int):
        out = np.zeros(3, dtype=np.uint64)
        lib().dox_get_indices(C.byref(self._m), C.c_uint64(cell), _p(out, C.c_uint64))
        return tuple(int(v) for v in out)

    def get_refinement_level(self, cell: int) -> int:
        return lib().dox_get_refinement_level(C.byref(self._m), C.c_uint64(cell))

    def get_cell_length_in_indices(self, cell: int) -> int:
        return lib().dox_get_cell_length_in_indices(C.byref(self._m), C.c_uint64(cell))

    def get_parent(self, cell: int) -> int:
        return lib().dox_get_parent(C.byref(self._m), C.c_uint64(cell))

    def get_child(self, cell: int) -> int:
        return lib().dox_get_child(C.byref(self._m), C.c_uint64(cell))

    def get_level_0_parent(self, cell: int) -> int:
        return lib().dox_get_level_0_parent(C.byref(self._m), C.c_uint64(cell))

    def get_all_children(self, cell: int):
        out = np.zeros(8, dtype=np.uint64)
        lib().dox_get_all_children(C.byref(self._m), C.c_uint64(cell), _p(out, C.c_uint64))
        return [int(v) for v in out]

    def get_siblings(self, cell: int):
        out = np.zeros(8, dtype=np.uint64)
        lib().dox_get_siblings(C.byref(self._m), C.c_uint64(cell), _p(out, C.c_uint64))
        return [int(v) for v in out]

    def ids_to_indices(self, ids: np.ndarray):
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        idx = np.zeros((ids.size, 3), dtype=np.uint64)
        lvl = np.zeros(ids.size, dtype=np.int32)
        lib().dox_map_ids_to_indices(C.byref(self._m), _p(ids, C.c_uint64), ids.size,
                                     _p(idx, C.c_uint64), _p(lvl, C.c_int32))
        return idx, lvl

    def indices_to_ids(self, idx: np.ndarray, lvl: np.ndarray) -> np.ndarray:
        idx = np.ascontiguousarray(idx, dtype=np.uint64).reshape(-1, 3)
        lvl = np.ascontiguousarray(lvl, dtype=np.int32)
        out = np.zeros(lvl.size, dtype=np.uint64)
        lib().dox_map_indices_to_ids(C.byref(self._m), _p(idx, C.c_uint64), _p(lvl, C.c_int32),
                                     lvl.size, _p(out, C.c_uint64))
        return out


def max_possible_refinement_level(length) -> int:
    ln = np.array(length, dtype=np.uint64)
    return lib().dox_max_possible_refinement_level(_p(ln, C.c_uint64))


def block_owner(total_cells: int, comm_size: int, level0_cell: int) -> int:
    """dccrg.hpp:8098-8145."""
    return lib().dox_block_owner(total_cells, comm_size, level0_cell)


def block_first_cell(total_cells: int, comm_size: int, rank: int) -> int:
    return lib().dox_block_first_cell(total_cells, comm_size, rank)


class Grid:
    """The set of existing leaf cells + the reference's neighbor algorithms."""

    def __init__(self, length, max_ref_lvl=0, periodic=(False, False, False), hood_length=1,
                 leaves=None):
        self.mapping = Mapping(length, max_ref_lvl)
        self.length = tuple(int(v) for v in length)
        self.periodic = tuple(bool(p) for p in periodic)
        self.hood_length = int(hood_length)
        ln = np.array(length, dtype=np.uint64)
        per = np.array(periodic, dtype=np.uint8)
        if leaves is None:
            h = lib().dox_grid_create(_p(ln, C.c_uint64), self.mapping.max_ref_lvl,
                                      _p(per, C.c_uint8), None, 0)
        else:
            lv = np.ascontiguousarray(leaves, dtype=np.uint64)
            h = lib().dox_grid_create(_p(ln, C.c_uint64), self.mapping.max_ref_lvl,
                                      _p(per, C.c_uint8), _p(lv, C.c_uint64), lv.size)
        if not h:
            raise ValueError("invalid grid")
        self._h = h
        self.hood_of = default_neighborhood(self.hood_length)
        self.hood_to = neighborhood_to(self.hood_of)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().dox_grid_destroy(h)
            self._h = None

    def cells(self) -> np.ndarray:
        n = lib().dox_grid_size(self._h)
        out = np.zeros(n, dtype=np.uint64)
        lib().dox_grid_cells(self._h, _p(out, C.c_uint64), n)
        return out

    def exists(self, cell: int) -> bool:
        return bool(lib().dox_grid_exists(self._h, C.c_uint64(cell)))

    def face_graph(self, cell: int):
        out = np.zeros(6, dtype=np.uint64)
        lib().dox_update_neighbors_(self._h, C.c_uint64(cell), _p(out, C.c_uint64))
        return [int(v) for v in out]

    def find_neighbors_of(self, cell: int, items=None) -> List[Tuple[int, Tuple[int, int, int]]]:
        items = self.hood_of if items is None else np.ascontiguousarray(items, dtype=np.int32)
        items = np.ascontiguousarray(items, dtype=np.int32).reshape(-1, 3)
        cap = 8 * len(items) + 8
        ids = np.zeros(cap, dtype=np.uint64)
        off = np.zeros((cap, 3), dtype=np.int32)
        n = lib().dox_find_neighbors_of(self._h, C.c_uint64(cell), _p(items, C.c_int32),
                                        len(items), _p(ids, C.c_uint64), _p(off, C.c_int32), cap)
        if n < 0:
            raise RuntimeError(f"find_neighbors_of({cell}) failed: {n}")
        return [(int(ids[i]), (int(off[i, 0]), int(off[i, 1]), int(off[i, 2]))) for i in range(n)]

    def find_neighbors_to(self, cell: int, items=None) -> List[int]:
        items = self.hood_to if items is None else np.ascontiguousarray(items, dtype=np.int32)
        items = np.ascontiguousarray(items, dtype=np.int32).reshape(-1, 3)
        cap = 16 * len(items) + 16
        ids = np.zeros(cap, dtype=np.uint64)
        n = lib().dox_find_neighbors_to(self._h, C.c_uint64(cell), _p(items, C.c_int32),
                                        len(items), _p(ids, C.c_uint64), cap)
        if n < 0:
            raise RuntimeError(f"find_neighbors_to({cell}) failed: {n}")
        return [int(v) for v in ids[:n]]

    def face_neighbors_of(self, cell: int) -> List[Tuple[int, int]]:
        ids = np.zeros(64, dtype=np.uint64)
        dirs = np.zeros(64, dtype=np.int32)
        n = lib().dox_get_face_neighbors_of(self._h, C.c_uint64(cell), _p(ids, C.c_uint64),
                                            _p(dirs, C.c_int32), 64)
        if n < 0:
            raise RuntimeError("face neighbors failed")
        return [(int(ids[i]), int(dirs[i])) for i in range(n)]

    # ---- per-rank bookkeeping (pure Python restatements) ------------------
    def owner(self, cell: int, comm_size: int) -> int:
        """Owner of a cell without load balancing: children stay on the process
        of their refinement-level-0 ancestor (dccrg.hpp:8116-8145 + refines in
        place, no migration under DCCRG_NO_LB).  ``self.l0_owner`` (a table
        from sfc_owner_table) replaces the block partition when set."""
        l0 = self.mapping.get_level_0_parent(cell)
        table = getattr(self, "l0_owner", None)
        if table is not None:
            return int(table[l0 - 1])
        total = self.length[0] * self.length[1] * self.length[2]
        return block_owner(total, comm_size, l0)

    def rank_view(self, rank: int, comm_size: int, items_of=None, items_to=None):
        """Everything one rank derives at initialize() time.

        local cells, neighbors_of / neighbors_to per local cell,
        local/remote cells on the process boundary (dccrg.hpp:9131-9234,
        9377-9409), per-peer sorted send/receive lists (dccrg.hpp:8729-8891).
        """
        items_of = self.hood_of if items_of is None else np.asarray(items_of, dtype=np.int32)
        items_to = neighborhood_to(items_of) if items_to is None else items_to
        local = [int(c) for c in self.cells() if self.owner(int(c), comm_size) == rank]
        nof: Dict[int, list] = {}
        nto: Dict[int, list] = {}
        local_bdy, remote_bdy = set(), set()
        send: Dict[int, set] = {}
        recv: Dict[int, set] = {}
        for c in local:
            nof[c] = self.find_neighbors_of(c, items_of)
            nto[c] = self.find_neighbors_to(c, items_to)
            for n, _ in nof[c]:
                p = self.owner(n, comm_size)
                if p != rank:
                    local_bdy.add(c)
                    remote_bdy.add(n)
                    recv.setdefault(p, set()).add(n)
            for n in nto[c]:
                p = self.owner(n, comm_size)
                if p != rank:
                    local_bdy.add(c)
                    remote_bdy.add(n)
                    send.setdefault(p, set()).add(c)
        return {
            "local": sorted(local),
            "neighbors_of": nof,
            "neighbors_to": nto,
            "inner": sorted(set(local) - local_bdy),
            "outer": sorted(local_bdy),
            "remote": sorted(remote_bdy),
            "send": {p: sorted(v) for p, v in send.items()},
            "recv": {p: sorted(v) for p, v in recv.items()},
        }


def iteration_cache_lists(nof: List[Tuple[int, Tuple[int, int, int]]], nto: List[int]):
    """Neighbor order in the iteration cache, dccrg.hpp:11570-11712.

    Returns (neighbors_of_range, neighbors_to_range) where each item is
    (id, (x, y, z)).  neighbors_of = [only_of][both], neighbors_to =
    [both][only_to]; each group is std::set-sorted by (id, offset).
    """
    ids_of = sorted(set((i, o) for i, o in nof if i != ERROR_CELL))
    ids_to = sorted(set((i, (0, 0, 0)) for i in nto if i != ERROR_CELL))
    only_to = set(ids_to)
    both, only_of = set(), set()
    to_set = set(ids_to)
    for n in ids_of:
        tmp = (n[0], (0, 0, 0))
        only_to.discard(tmp)
        if tmp in to_set:
            both.add(n)
        else:
            only_of.add(n)
    only_of, both, only_to = sorted(only_of), sorted(both), sorted(only_to)
    return only_of + both, both + only_to


def gol_reference_run(length, periodic, hood_length, alive0: np.ndarray, steps: int):
    """Uniform level-0 grid, game of life with the reference's rule over the
    reference's neighbors_of lists (face-graph walk).  alive0 is indexed by
    cell id - 1.  Returns (alive, live_neighbor_count) after ``steps``."""
    g = Grid(length, 0, periodic, hood_length)
    n = int(np.prod(length))
    k = len(g.hood_of)
    row_ptr = np.zeros(n + 1, dtype=np.uint64)
    cap = n * k
    slots = np.zeros(cap, dtype=np.uint32)
    tot = lib().dox_build_uniform_slot_lists(g._h, hood_length, _p(row_ptr, C.c_uint64),
                                             _p(slots, C.c_uint32), cap)
    if tot < 0:
        raise RuntimeError("slot list build failed")
    alive = np.ascontiguousarray(alive0, dtype=np.uint32).copy()
    count = np.zeros(n, dtype=np.uint32)
    for _ in range(steps):
        lib().dox_gol_count(n, _p(row_ptr, C.c_uint64), _p(slots, C.c_uint32),
                            _p(alive, C.c_uint32), _p(count, C.c_uint32))
        lib().dox_gol_apply(n, _p(alive, C.c_uint32), _p(count, C.c_uint32))
    return alive, count


class GolLists:
    """Pre-built explicit lists for repeated stepping (cpu_baseline)."""

    def __init__(self, length, periodic, hood_length):
        self.grid = Grid(length, 0, periodic, hood_length)
        self.n = int(np.prod(length))
        k = len(self.grid.hood_of)
        self.row_ptr = np.zeros(self.n + 1, dtype=np.uint64)
        self.slots = np.zeros(self.n * k, dtype=np.uint32)
        tot = lib().dox_build_uniform_slot_lists(self.grid._h, hood_length,
                                                 _p(self.row_ptr, C.c_uint64),
                                                 _p(self.slots, C.c_uint32), self.n * k)
        if tot < 0:
            raise RuntimeError("slot list build failed")

    def step(self, alive: np.ndarray, count: np.ndarray):
        lib().dox_gol_count(self.n, _p(self.row_ptr, C.c_uint64), _p(self.slots, C.c_uint32),
                            _p(alive, C.c_uint32), _p(count, C.c_uint32))
        lib().dox_gol_apply(self.n, _p(alive, C.c_uint32), _p(count, C.c_uint32))


def splitmix64(x: np.ndarray) -> np.ndarray:
    """Seed function for reproducible random initial states."""
    with np.errstate(over="ignore"):
        z = (np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def random_alive(ids: np.ndarray, p_permille: int = 200) -> np.ndarray:
    """alive = splitmix64(id) % 1000 < p_permille (bit-exact on CPU and GPU)."""
    return (splitmix64(ids) % np.uint64(1000) < np.uint64(p_permille)).astype(np.uint32)


def random_balanced_leaves(length, max_ref_lvl, periodic, hood_length, n_refines, seed):
    """Random 2:1-balanced leaf set (test input generator): a cell of level l
    is refined only when every cell in its neighbors_of and neighbors_to has
    level >= l, which keeps neighbors within one level (the assumption of
    dccrg.hpp:4736-4737, enforced in the reference by induce_refines)."""
    rng = np.random.default_rng(seed)
    m = Mapping(length, max_ref_lvl)
    cells = set(range(1, int(np.prod(length)) + 1))
    for _ in range(n_refines):
        g = Grid(length, max_ref_lvl, periodic, hood_length, sorted(cells))
        cand = sorted(c for c in cells if m.get_refinement_level(c) < m.max_ref_lvl)
        if not cand:
            break
        c = int(cand[int(rng.integers(len(cand)))])
        lvl = m.get_refinement_level(c)
        if all(m.get_refinement_level(n) >= lvl for n, _ in g.find_neighbors_of(c)) and \
                all(m.get_refinement_level(n) >= lvl for n in g.find_neighbors_to(c)):
            cells.discard(c)
            cells |= set(m.get_all_children(c))
    return sorted(cells)


# ---- advection (tests/advection) --------------------------------------------
def advection_initial_state(mapping: Mapping, cells: Sequence[int], level0_length=None):
    """tests/advection/initialize.hpp:27-65 on a Cartesian geometry starting
    at 0 with level-0 cell length ``level0_length`` (default 1 / length per
    axis): hump density, solid-body velocities (solve.hpp:335-345), cell
    lengths.  Returns slot-ordered (density, vx, vy, vz, lx, ly, lz)."""
    L = mapping.length
    l0 = np.array(level0_length if level0_length is not None else [1.0 / x for x in L])
    M = mapping.max_ref_lvl
    cells = np.asarray(cells, dtype=np.uint64)
    idx, lvl = mapping.ids_to_indices(cells)
    unit = l0 / float(2 ** M)
    ln = l0[None, :] / (2.0 ** lvl.astype(np.float64))[:, None]
    center = idx.astype(np.float64) * unit[None, :] + ln / 2
    r = np.minimum(np.sqrt((center[:, 0] - 0.25) ** 2 + (center[:, 1] - 0.5) ** 2), 0.15) / 0.15
    density = 0.25 * (1 + np.cos(np.pi * r))
    vx = -center[:, 1] + 0.5
    vy = center[:, 0] - 0.5
    vz = np.zeros(len(cells))
    return [np.ascontiguousarray(a, dtype=np.float64)
            for a in (density, vx, vy, vz, ln[:, 0], ln[:, 1], ln[:, 2])]


class AdvectionLists:
    """The reference advection solver (solve.hpp:44-332) on every rank of a
    block-partitioned grid, over the iteration-cache neighbor lists
    (dccrg.hpp:11570-11712).  Slots = positions in ``cells`` (ascending)."""

    def __init__(self, grid: "Grid", comm_size: int = 1, items=None):
        self.cells = [int(c) for c in grid.cells()]
        pos = {c: i for i, c in enumerate(self.cells)}
        m = grid.mapping
        n = len(self.cells)
        self.n = n
        self.len_idx = np.array([m.get_cell_length_in_indices(c) for c in self.cells], dtype=np.uint64)
        self.ranks = []
        for r in range(comm_size):
            v = grid.rank_view(r, comm_size, items)
            is_local = np.zeros(n, dtype=np.uint8)
            local = np.array([pos[c] for c in v["local"]], dtype=np.uint32)
            is_local[local] = 1
            order = v["inner"] + v["outer"]  # 2d.cpp:331 then :339
            row = [0]
            slots, offs = [], []
            for c in order:
                lof, _ = iteration_cache_lists(v["neighbors_of"][c], v["neighbors_to"][c])
                for i, o in lof:
                    slots.append(pos[i])
                    offs.extend(o)
                row.append(len(slots))
            self.ranks.append({
                "iter": np.array([pos[c] for c in order], dtype=np.uint32),
                "row": np.array(row, dtype=np.uint64),
                "slots": np.array(slots or [0], dtype=np.uint32),
                "offs": np.array(offs or [0, 0, 0], dtype=np.int32),
                "is_local": is_local,
                "local": local,
            })

    def step(self, state, dt: float):
        """One 2d.cpp:321-390 step on every rank; returns the new density."""
        rho, vx, vy, vz, lx, ly, lz = state
        new = rho.copy()
        f64 = C.c_double
        for R in self.ranks:
            flux = np.zeros(self.n)
            bad = lib().dox_advect_fluxes(
                len(R["iter"]), _p(R["iter"], C.c_uint32), _p(R["row"], C.c_uint64),
                _p(R["slots"], C.c_uint32), _p(R["offs"], C.c_int32), _p(R["is_local"], C.c_uint8),
                _p(self.len_idx, C.c_uint64), _p(rho, f64), _p(vx, f64), _p(vy, f64), _p(vz, f64),
                _p(lx, f64), _p(ly, f64), _p(lz, f64), _p(flux, f64), dt)
            if bad:
                raise RuntimeError("overlapping neighbor (solve.hpp:101-116 aborts)")
            mine = rho.copy()
            lib().dox_advect_apply(len(R["local"]), _p(R["local"], C.c_uint32), _p(mine, f64), _p(flux, f64))
            new[R["local"]] = mine[R["local"]]
        return new

    def max_time_step(self, state) -> float:
        """solve.hpp:302-332 including the MIN reduction over ranks."""
        _, vx, vy, vz, lx, ly, lz = state
        f64 = C.c_double
        return min(lib().dox_advect_max_time_step(len(R["local"]), _p(R["local"], C.c_uint32), _p(vx, f64),
                                                  _p(vy, f64), _p(vz, f64), _p(lx, f64), _p(ly, f64),
                                                  _p(lz, f64)) for R in self.ranks)


# ---- Poisson (tests/poisson/poisson_solve.hpp) -------------------------------
POISSON_SOLVE, POISSON_BOUNDARY, POISSON_SKIP = 0.0, 1.0, 2.0  # :160-165


class PoissonSystem:
    """Poisson_Solve's cached system (cache_system_info, poisson_solve.hpp:
    827-971, set_scaling_factor :704-821) on every rank of a block-partitioned
    grid, and solve() via the C restatement.  Slots = positions in
    ``grid.cells()``.  ``lengths`` = (lx, ly, lz) slot arrays (the geometry's
    get_length).  Cell order within a rank: ascending id (the reference's
    get_cells() order is its hash order; only sums' order depends on it)."""

    def __init__(self, grid: "Grid", comm_size: int, lengths, solve_cells=None, skip_cells=()):
        self.cells = [int(c) for c in grid.cells()]
        pos = {c: i for i, c in enumerate(self.cells)}
        n = len(self.cells)
        m = grid.mapping
        solve = set(self.cells if solve_cells is None else solve_cells)
        skip = set(skip_cells) - solve
        owner = [grid.owner(c, comm_size) for c in self.cells]
        self.type = np.full(n, POISSON_BOUNDARY)
        for c in skip:
            self.type[pos[c]] = POISSON_SKIP
        for c in solve:
            self.type[pos[c]] = POISSON_SOLVE
        lx, ly, lz = (np.asarray(a, dtype=np.float64) for a in lengths)
        self.f = np.zeros((n, 6))
        self.sf = np.zeros(n)
        info, row, nb, code, rank_begin = [], [0], [], [], [0]
        for r in range(comm_size):
            for c in self.cells:
                i = pos[c]
                if owner[i] != r or self.type[i] == POISSON_SKIP:
                    continue
                lvl = m.get_refinement_level(c)
                kept = []
                for nbr, d in grid.face_neighbors_of(c):
                    j = pos[nbr]
                    if self.type[j] == POISSON_SKIP:
                        continue
                    if self.type[i] == POISSON_BOUNDARY and self.type[j] == POISSON_BOUNDARY:
                        continue
                    nl = m.get_refinement_level(nbr)
                    rel = 1 if nl > lvl else (-1 if nl < lvl else 0)
                    kept.append((j, d, rel))
                if not kept:
                    self.type[i] = POISSON_SKIP
                    continue
                self._scaling(i, kept, lx, ly, lz)
                info.append(i)
                for j, d, rel in kept:
                    nb.append(j)
                    code.append((d + 3) | ((rel + 1) << 4))
                row.append(len(nb))
            rank_begin.append(len(info))
        self.info = np.array(info, dtype=np.uint32)
        self.row = np.array(row, dtype=np.uint64)
        self.nb = np.array(nb or [0], dtype=np.uint32)
        self.code = np.array(code or [0], dtype=np.int32)
        self.rank_begin = np.array(rank_begin, dtype=np.uintp)
        self.P = comm_size

    def _scaling(self, i, kept, lx, ly, lz):
        """set_scaling_factor, poisson_solve.hpp:704-821."""
        hx, hy, hz = lx[i] / 2.0, ly[i] / 2.0, lz[i] / 2.0
        pos_x, neg_x = +2 * hx, -2 * hx
        pos_y, neg_y = +2 * hy, -2 * hy
        pos_z, neg_z = +2 * hz, -2 * hz
        for j, d, _ in kept:
            nx, ny, nz = lx[j] / 2.0, ly[j] / 2.0, lz[j] / 2.0
            if d == 1:
                pos_x = hx + nx
            elif d == -1:
                neg_x = -1.0 * (hx + nx)
            elif d == 2:
                pos_y = hy + ny
            elif d == -2:
                neg_y = -1.0 * (hy + ny)
            elif d == 3:
                pos_z = hz + nz
            else:
                neg_z = -1.0 * (hz + nz)
        tx, ty, tz = pos_x - neg_x, pos_y - neg_y, pos_z - neg_z
        f = [0.0] * 6
        for _, d, _ in kept:
            if d == 1:
                f[0] = +2.0 / (pos_x * tx)
            elif d == -1:
                f[1] = -2.0 / (neg_x * tx)
            elif d == 2:
                f[2] = +2.0 / (pos_y * ty)
            elif d == -2:
                f[3] = -2.0 / (neg_y * ty)
            elif d == 3:
                f[4] = +2.0 / (pos_z * tz)
            else:
                f[5] = -2.0 / (neg_z * tz)
        self.f[i] = f
        self.sf[i] = -f[0] - f[1] - f[2] - f[3] - f[4] - f[5]

    def solve(self, rhs, solution, max_iterations=1000, min_iterations=0, stop_residual=1e-15,
              p_of_norm=2.0, stop_after_residual_increase=10.0):
        """Poisson_Solve::solve (:251-522).  Returns (solution, iterations,
        minimum residual); ``solution`` holds the initial guess."""
        n = len(self.cells)
        f64 = C.c_double
        sol = np.ascontiguousarray(solution, dtype=np.float64).copy()
        rhs = np.ascontiguousarray(rhs, dtype=np.float64)
        work = [np.zeros(n) for _ in range(7)]  # best, p0, p1, r0, r1, adp0
        res = C.c_double()
        f = np.ascontiguousarray(self.f)
        it = lib().dox_poisson_solve(
            len(self.info), _p(self.info, C.c_uint32), self.P,
            self.rank_begin.ctypes.data_as(C.POINTER(C.c_size_t)), _p(self.row, C.c_uint64),
            _p(self.nb, C.c_uint32), _p(self.code, C.c_int32), _p(self.type, f64), _p(rhs, f64), _p(sol, f64),
            *[_p(w, f64) for w in work[:6]], _p(self.sf, f64), _p(f, f64), max_iterations, min_iterations,
            stop_residual, p_of_norm, stop_after_residual_increase, C.byref(res))
        if it < 0:
            raise RuntimeError("dox_poisson_solve failed")
        return sol, int(it), res.value


# ---- AMR-aware game of life (tests/game_of_life/solve.hpp) -------------------
class GolHierarchical:
    """tests/game_of_life/solve.hpp:40-170 (= solve_optimized.hpp:40-133) on
    every rank of a block-partitioned grid, restated literally.  A cell is
    ``Cell::data`` = 9 x u64 (tests/game_of_life/cell.hpp:32-47): data[0] the
    state, data[1..8] the level-0 parents of live neighbors.  One call of
    ``get_live_neighbors`` is: (1) every local cell records the distinct
    level-0 parents of its live neighbors_of entries (own parent skipped, in
    list order), (2) update_copies_of_remote_neighbors, (3) in ``order`` each
    local cell merges the lists of neighbors sharing its level-0 parent (the
    CURRENT lists: earlier merges of this phase are seen, as the reference's
    sequential loop sees them), (4) B3/S23 on the number of recorded parents
    and the lists reset to error_cell.  The reference aborts when a list
    overflows or a dead neighbor's parent is already recorded: raised here.
    ``halo()`` is the caller's update before each call
    (game_of_life_test.cpp:378-380)."""

    def __init__(self, grid: "Grid", comm_size: int = 1):
        self.grid = grid
        self.P = comm_size
        self.cells = [int(c) for c in grid.cells()]
        m = grid.mapping
        self.par = {c: m.get_level_0_parent(c) for c in self.cells}
        self.owner = {c: grid.owner(c, comm_size) for c in self.cells}
        self.nof = {c: [n for n, _ in grid.find_neighbors_of(c)] for c in self.cells}
        self.data = {c: [0] * 9 for c in self.cells}
        self.ghost = [dict() for _ in range(comm_size)]

    def halo(self):
        """update_copies_of_remote_neighbors on every rank."""
        for c in self.cells:
            r = self.owner[c]
            for n in self.nof[c]:
                if n != ERROR_CELL and self.owner[n] != r:
                    self.ghost[r][n] = list(self.data[n])

    def _d(self, rank: int, cell: int):
        return self.data[cell] if self.owner[cell] == rank else self.ghost[rank][cell]

    def get_live_neighbors(self, order: str = "ascending"):
        for c in self.cells:  # phase 1 (independent per cell)
            r, d = self.owner[c], self.data[c]
            for i in range(1, 9):
                d[i] = 0
            for n in self.nof[c]:
                if n == ERROR_CELL or self.par[n] == self.par[c]:
                    continue
                pn = self.par[n]
                if self._d(r, n)[0] == 0:
                    if pn in d[1:]:
                        raise RuntimeError(f"neighbor {n} of cell {c} should not be alive")
                    continue
                for i in range(1, 9):
                    if d[i] == pn:
                        break
                    if d[i] == ERROR_CELL:
                        d[i] = pn
                        break
                    if i == 8:
                        raise OverflowError("No more room in live neighbor list")
        self.halo()
        seq = sorted(self.cells, reverse=(order == "descending"))
        for c in seq:  # phase 2 (sequential per rank; siblings share the rank)
            r, d = self.owner[c], self.data[c]
            for n in self.nof[c]:
                if n == ERROR_CELL or self.par[n] != self.par[c]:
                    continue
                nd = self._d(r, n)
                for i in range(1, 9):
                    if nd[i] == ERROR_CELL:
                        break
                    for j in range(1, 9):
                        if d[j] == ERROR_CELL:
                            d[j] = nd[i]
                            break
                        if d[j] == nd[i]:
                            break
                        if j == 8:
                            raise OverflowError("No room in live neighbor list")
        for c in self.cells:  # phase 3
            d = self.data[c]
            live = sum(1 for i in range(1, 9) if d[i] != ERROR_CELL)
            for i in range(1, 9):
                d[i] = ERROR_CELL
            if live == 3:
                d[0] = 1
            elif live != 2:
                d[0] = 0

    def alive(self) -> np.ndarray:
        return np.array([self.data[c][0] for c in self.cells], dtype=np.uint64)


# ---- space-filling-curve placement (dccrg.hpp:8147-8220, USE_SFC) -----------
def hilbert_keys(length) -> np.ndarray:
    """Hilbert index of every level-0 cell (index id - 1): Skilling's
    axes-to-transpose (AIP Conf. Proc. 707, 2004) with b bits per axis, the
    smallest power of two >= the longest side, x = X[0]; the transpose is
    read out most significant bit first, X[0] X[1] X[2] per bit.  Restated
    independently of sfc.hip (numpy, vectorised over cells)."""
    L = [int(v) for v in length]
    n = L[0] * L[1] * L[2]
    side = max(L)
    b = 1
    while (1 << b) < side:
        b += 1
    lin = np.arange(n, dtype=np.uint64)
    X = [lin % np.uint64(L[0]), (lin // np.uint64(L[0])) % np.uint64(L[1]), lin // np.uint64(L[0] * L[1])]
    M = 1 << (b - 1)
    Q = M
    while Q > 1:
        P = np.uint64(Q - 1)
        q = np.uint64(Q)
        for i in range(3):
            hit = (X[i] & q) != 0
            t = (X[0] ^ X[i]) & P
            X[0] = np.where(hit, X[0] ^ P, X[0] ^ t)
            if i:
                X[i] = np.where(hit, X[i], X[i] ^ t)
        Q >>= 1
    X[1] = X[1] ^ X[0]
    X[2] = X[2] ^ X[1]
    t = np.zeros(n, dtype=np.uint64)
    Q = M
    while Q > 1:
        t = np.where((X[2] & np.uint64(Q)) != 0, t ^ np.uint64(Q - 1), t)
        Q >>= 1
    X = [x ^ t for x in X]
    key = np.zeros(n, dtype=np.uint64)
    for bit in range(b - 1, -1, -1):
        for i in range(3):
            key = (key << np.uint64(1)) | ((X[i] >> np.uint64(bit)) & np.uint64(1))
    return key


def sfc_owner_table(length, comm_size: int) -> np.ndarray:
    """create_level_0_cells with USE_SFC (dccrg.hpp:8147-8220): the cells in
    curve order get the block partition's per-process counts (:8098-8114)."""
    key = hilbert_keys(length)
    order = np.argsort(key, kind="stable")
    n = key.size
    cpp = 1 if n < comm_size else (n // comm_size + (1 if n % comm_size else 0))
    fewer = cpp * comm_size - n
    pos = np.arange(n, dtype=np.int64)
    split = fewer * (cpp - 1)
    owner_of_pos = np.where(pos < split, pos // max(cpp - 1, 1), fewer + (pos - split) // cpp)
    table = np.empty(n, dtype=np.int32)
    table[order] = owner_of_pos
    return table
