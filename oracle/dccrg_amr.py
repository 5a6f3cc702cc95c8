"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's AMR control
logic (refine / unrefine requests, their overrides and inductions, and the
leaf-set update of execute_refines), used as the checker of the library's
stop_refining.  Only ``tests/`` may import it.

Follows dccrg.hpp line by line, with every rank of a P-process run simulated
in one process (the All_Gather / All_Reduce calls become loops over the
simulated ranks):
  - refine_completely      :2456-2548
  - unrefine_completely    :2582-2676
  - dont_unrefine          :2701-2760
  - dont_refine            :2768-2806
  - stop_refining          :3483-3507 = override_refines :10130-10236,
                             induce_refines :9730-9907, override_unrefines
                             :9935-10124, execute_refines :10243-10693
  - get_removed_cells      :3519-3543
  - is_neighbor            :9603-9683, overlapping_indices :11364-11405
Neighbor lists (neighbors_of / neighbors_to of every cell) and the face graph
(neighbors_, update_neighbors_) come from the oracle's C restatement of the
face-graph walk (dccrg_oracle.c), rebuilt after every execution as the
reference rebuilds them (:10642-10690).

One documented deviation: unrefine_completely calls
find_neighbors_of(parent, ...) (:2638-2639) for the parent of the cell, which
is not in cell_process and makes find_neighbors_of throw (:4390-4398).  The
documented intent (:2561-2580, "unrefinement succeeds if parent of unrefined
will fulfill requirements") is restated instead: the leaves overlapping the
parent's neighborhood windows are inspected.

Ownership without load balancing: every cell stays on the process of its
refinement-level-0 ancestor (children are created on the parent's process,
:10368; the parent of unrefined cells goes to the owner of its first child,
:10437), i.e. the block partition of level-0 cells (:8116-8145).

Parity pinning: the reference's own refinement tests (tests/refine/
dont_refine.cpp, refine_simple.cpp, unrefine_simple.cpp) state their expected
outcomes in code; tests/test_oracle_amr.py replays them against this module.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Set

import numpy as np

from oracle.dccrg_oracle import Grid, Mapping, block_owner, default_neighborhood

ERROR_CELL = 0


class AmrOracle:
    def __init__(self, length, max_ref_lvl, periodic=(False, False, False), hood_length=1, comm_size=1,
                 leaves: Optional[Sequence[int]] = None, l0_owner=None):
        """l0_owner: owner table of the level-0 cells (SFC placement,
        dccrg_oracle.sfc_owner_table); None = the block partition."""
        self.l0_owner = l0_owner
        self.length = tuple(int(v) for v in length)
        self.mapping = Mapping(self.length, max_ref_lvl)
        self.M = self.mapping.max_ref_lvl
        self.periodic = tuple(bool(p) for p in periodic)
        self.hood_length = int(hood_length)
        self.P = int(comm_size)
        self.N0 = self.length[0] * self.length[1] * self.length[2]
        if leaves is None:
            leaves = range(1, self.N0 + 1)
        self.leaves: Set[int] = set(int(c) for c in leaves)
        self.items = default_neighborhood(self.hood_length)
        self._rebuild()
        # per-rank request state (dccrg.hpp:7355-7360)
        self.to_refine = [set() for _ in range(self.P)]
        self.not_to_refine = [set() for _ in range(self.P)]
        self.to_unrefine = [set() for _ in range(self.P)]
        self.not_to_unrefine = [set() for _ in range(self.P)]
        self.removed: List[List[int]] = [[] for _ in range(self.P)]

    # ---- structure ---------------------------------------------------------
    def _rebuild(self):
        self.grid = Grid(self.length, self.M, self.periodic, self.hood_length, sorted(self.leaves))
        self.grid.l0_owner = self.l0_owner
        self._nof: Dict[int, List[int]] = {}
        self._nto: Dict[int, List[int]] = {}
        self._bdy = None

    def level(self, c: int) -> int:
        return self.mapping.get_refinement_level(c)

    def exists(self, c: int) -> bool:
        return c in self.leaves

    def owner(self, c: int) -> int:
        l0 = self.mapping.get_level_0_parent(c)
        if self.l0_owner is not None:
            return int(self.l0_owner[l0 - 1])
        return block_owner(self.N0, self.P, l0)

    def nof(self, c: int) -> List[int]:
        if c not in self._nof:
            self._nof[c] = [n for n, _ in self.grid.find_neighbors_of(c)]
        return self._nof[c]

    def nto(self, c: int) -> List[int]:
        if c not in self._nto:
            self._nto[c] = self.grid.find_neighbors_to(c)
        return self._nto[c]

    def face(self, c: int) -> List[int]:
        return self.grid.face_graph(c)

    def siblings(self, c: int) -> List[int]:
        return self.mapping.get_siblings(c)

    def has_children(self, c: int) -> bool:
        """c != get_child(c) (dccrg.hpp:9694-9718) for a cell that exists or not."""
        if self.level(c) == self.M:
            return c not in self.leaves
        child = self.mapping.get_child(c)
        if child in self.leaves:
            return True
        return c not in self.leaves

    def boundary(self, rank: int):
        """local / remote cells on the process boundary of the default
        neighborhood (dccrg.hpp:9131-9234)."""
        if self._bdy is None:
            self._bdy = {}
        if rank not in self._bdy:
            loc, rem = set(), set()
            for c in self.leaves:
                if self.owner(c) != rank:
                    continue
                for n in self.nof(c) + self.nto(c):
                    if self.owner(n) != rank:
                        loc.add(c)
                        rem.add(n)
            self._bdy[rank] = (loc, rem)
        return self._bdy[rank]

    def is_neighbor(self, cell1: int, cell2: int) -> bool:
        """dccrg.hpp:9603-9683."""
        m = self.mapping
        i1, i2 = m.get_indices(cell1), m.get_indices(cell2)
        l1, l2 = m.get_cell_length_in_indices(cell1), m.get_cell_length_in_indices(cell2)
        glen = [self.length[d] << self.M for d in range(3)]
        maxd = 0
        for d in range(3):
            if i1[d] <= i2[d]:
                dist = 0 if i2[d] <= i1[d] + l1 else i2[d] - (i1[d] + l1)
                if self.periodic[d]:
                    dist = min(dist, i1[d] + (glen[d] - (i2[d] + l2)))
            else:
                dist = 0 if i1[d] <= i2[d] + l2 else i1[d] - (i2[d] + l2)
                if self.periodic[d]:
                    dist = min(dist, i2[d] + (glen[d] - (i1[d] + l1)))
            maxd = max(maxd, dist)
        if self.hood_length == 0:
            return maxd < l1 and self.overlapping_indices(cell1, cell2) >= 2
        return maxd < self.hood_length * l1

    def overlapping_indices(self, cell1: int, cell2: int) -> int:
        """dccrg.hpp:11364-11405 + indices_overlap :11217-11254."""
        m = self.mapping
        i1, i2 = m.get_indices(cell1), m.get_indices(cell2)
        s1, s2 = m.get_cell_length_in_indices(cell1), m.get_cell_length_in_indices(cell2)
        return sum(1 for d in range(3) if i1[d] + s1 > i2[d] and i1[d] < i2[d] + s2)

    def parent_window_leaves(self, parent: int) -> List[int]:
        """Leaves overlapping the neighborhood windows of a (non-existing)
        parent cell -- the intent of find_neighbors_of(parent) in
        unrefine_completely (see the module docstring)."""
        m = self.mapping
        pl = self.level(parent)
        L = m.get_cell_length_in_indices(parent)
        pi = m.get_indices(parent)
        out = []

        def descend(w: int):
            if w in self.leaves:
                out.append(w)
                return
            if self.level(w) >= self.M:
                return
            for ch in m.get_all_children(w):
                descend(ch)

        for h in self.items:
            wi = []
            ok = True
            for d in range(3):
                G = self.length[d] << self.M
                x = pi[d] + int(h[d]) * L
                if x < 0 or x >= G:
                    if not self.periodic[d]:
                        ok = False
                        break
                    x %= G
                wi.append(x)
            if not ok:
                continue
            W = m.get_cell_from_indices(wi, pl)
            if W in self.leaves:
                out.append(W)
                continue
            if pl > 0:
                Pw = m.get_cell_from_indices(wi, pl - 1)
                if Pw in self.leaves:
                    out.append(Pw)
                    continue
            descend(W)
        return out

    # ---- requests (rank-local) ---------------------------------------------
    def refine_completely(self, rank: int, cell: int) -> bool:
        """dccrg.hpp:2456-2548."""
        if cell == ERROR_CELL or cell not in self.leaves or self.owner(cell) != rank:
            return False
        lvl = self.level(cell)
        if lvl == self.M:
            self.dont_unrefine(rank, cell)
            return True
        if cell in self.not_to_refine[rank]:
            return False
        for n in self.nof(cell):
            if self.level(n) < lvl and n in self.not_to_refine[rank]:
                return False
        self.to_refine[rank].add(cell)
        for s in self.siblings(cell):
            if s != ERROR_CELL:
                self.to_unrefine[rank].discard(s)
        for n in self.nof(cell) + self.nto(cell):
            if self.level(n) <= lvl:
                for s in self.siblings(n):
                    if s != ERROR_CELL:
                        self.to_unrefine[rank].discard(s)
        return True

    def unrefine_completely(self, rank: int, cell: int) -> bool:
        """dccrg.hpp:2582-2676."""
        if cell == ERROR_CELL or cell not in self.leaves or self.owner(cell) != rank:
            return False
        if self.level(cell) == 0:
            return True
        sibs = self.siblings(cell)
        for s in sibs:
            if self.has_children(s):
                return False
            if s in self.to_refine[rank] or s in self.not_to_unrefine[rank]:
                return True
        parent = self.mapping.get_parent(cell)
        plvl = self.level(parent)
        for n in self.parent_window_leaves(parent):
            nl = self.level(n)
            if nl > plvl + 1:
                return True
            if nl == plvl + 1 and n in self.to_refine[rank]:
                return True
        for s in sibs:
            if s in self.to_unrefine[rank]:
                return True
        self.to_unrefine[rank].add(cell)
        return True

    def dont_unrefine(self, rank: int, cell: int) -> bool:
        """dccrg.hpp:2701-2760."""
        if cell == ERROR_CELL or cell not in self.leaves:
            return False
        if self.level(cell) == 0:
            return True
        sibs = self.siblings(cell)
        if any(s in self.not_to_unrefine[rank] for s in sibs):
            return True
        for s in sibs:
            self.to_unrefine[rank].discard(s)
        self.not_to_unrefine[rank].add(cell)
        return True

    def dont_refine(self, rank: int, cell: int) -> bool:
        """dccrg.hpp:2768-2806."""
        if cell == ERROR_CELL or cell not in self.leaves:
            return False
        if self.level(cell) == self.M:
            return True
        self.to_refine[rank].discard(cell)
        self.not_to_refine[rank].add(cell)
        return True

    # ---- collective --------------------------------------------------------
    def _override_refines(self):
        """dccrg.hpp:10130-10236 (per rank; all_to_all_set = union)."""
        P = self.P
        new_donts = [set() for _ in range(P)]
        old_donts = [set() for _ in range(P)]
        while True:
            gathered = set()
            for r in range(P):
                donts = set(new_donts[r]) | self.not_to_refine[r]
                self.not_to_refine[r] = set()
                nd = set()
                for cell in donts:
                    allnb = set(self.nof(cell)) | set(self.nto(cell)) if cell in self.leaves else set()
                    rl = self.level(cell)
                    for n in allnb:
                        if n in old_donts[r] or n in donts:
                            continue
                        if self.level(n) > rl:
                            nd.add(n)
                old_donts[r] |= donts
                gathered |= nd
            new_donts = [set(gathered) for _ in range(P)]
            if not gathered:
                break
        nnr = set().union(*old_donts)
        for r in range(P):
            self.not_to_refine[r] = set(nnr)
            self.to_refine[r] -= nnr
        allr = set().union(*self.to_refine)
        for r in range(P):
            self.to_refine[r] = set(allr)

    def _induce_refines(self):
        """dccrg.hpp:9730-9907 (per rank)."""
        P = self.P
        new = [sorted(self.to_refine[r]) for r in range(P)]
        while sum(len(x) for x in new) > 0:
            all_new = [list(x) for x in new]
            new = [[] for _ in range(P)]
            for r in range(P):
                induced = set()
                for refined in all_new[r]:
                    rl = self.level(refined)
                    for n in self.nof(refined) + self.nto(refined):
                        if n == ERROR_CELL or self.owner(n) != r:
                            continue
                        if self.level(n) < rl and n not in self.to_refine[r]:
                            induced.add(n)
                loc_bdy, rem_bdy = self.boundary(r)
                for p in range(P):
                    if p == r:
                        continue
                    for refined in all_new[p]:
                        if refined not in rem_bdy:
                            continue
                        for local in loc_bdy:
                            if self.is_neighbor(local, refined) and self.level(local) < self.level(refined) \
                                    and local not in self.to_refine[r]:
                                induced.add(local)
                new[r] = sorted(induced)
                self.to_refine[r] |= induced
        allr = set().union(*self.to_refine)
        for r in range(P):
            self.to_refine[r] = set(allr)

    def _override_unrefines(self):
        """dccrg.hpp:9935-10124 (per rank)."""
        P = self.P
        nnu = set().union(*self.not_to_unrefine)
        R = self.to_refine[0]
        final = set()
        for r in range(P):
            for unrefined in self.to_unrefine[r]:
                parent = self.mapping.get_parent(unrefined)
                if any(s != ERROR_CELL and (s in R or s in nnu) for s in self.mapping.get_all_children(parent)):
                    continue
                ul = self.level(unrefined)
                can = True
                processed: Set[int] = set()
                process = set(self.face(unrefined))
                process.discard(ERROR_CELL)
                while process:
                    nxt = min(process)  # std::set iteration order
                    processed.add(nxt)
                    process.discard(nxt)
                    for n in self.face(nxt):
                        if n == ERROR_CELL or n in processed:
                            continue
                        if self.is_neighbor(parent, n):
                            process.add(n)
                        else:
                            processed.add(n)
                    rl = self.level(nxt)
                    if rl < ul:
                        continue
                    if rl == ul:
                        if nxt in R:
                            can = False
                            break
                        continue
                    can = False
                    break
                if can:
                    final.add(unrefined)
        for r in range(P):
            self.to_unrefine[r] = set(final)
            self.not_to_unrefine[r] = set()

    def _execute_refines(self) -> List[List[int]]:
        """dccrg.hpp:10243-10693: the leaf-set update; returns per-rank new
        cells (children of refined local cells) and records per-rank removed
        cells (siblings of unrefined cells whose parent is local)."""
        P = self.P
        R = set(self.to_refine[0])
        U = set(self.to_unrefine[0])
        new_cells = [[] for _ in range(P)]
        leaves = set(self.leaves)
        for refined in R:
            kids = self.mapping.get_all_children(refined)
            leaves.discard(refined)
            leaves |= set(kids)
            new_cells[self.owner(refined)].extend(kids)
        all_un = set()
        parents = set()
        for u in U:
            p = self.mapping.get_parent(u)
            parents.add(p)
            all_un |= set(self.mapping.get_all_children(p))
        self.removed = [[] for _ in range(P)]
        for u in all_un:
            leaves.discard(u)
            self.removed[self.owner(u)].append(u)
        leaves |= parents
        self.leaves = leaves
        for r in range(P):
            self.to_refine[r] = set()
            self.to_unrefine[r] = set()
            self.removed[r].sort()
            new_cells[r].sort()
        self._rebuild()
        return new_cells

    def stop_refining(self) -> List[List[int]]:
        """dccrg.hpp:3483-3507: per-rank new cells (sorted)."""
        self._override_refines()
        self._induce_refines()
        self._override_unrefines()
        return self._execute_refines()

    def get_removed_cells(self, rank: int) -> List[int]:
        return list(self.removed[rank])

    def cells(self) -> List[int]:
        return sorted(self.leaves)

    def max_level_difference(self) -> int:
        """Largest refinement level difference between a cell and any cell
        of its neighbors_of (the check of tests/refine/refine_simple.cpp)."""
        worst = 0
        for c in self.leaves:
            for n in self.nof(c):
                worst = max(worst, abs(self.level(c) - self.level(n)))
        return worst


# ---- the advection program with adaptation (tests/advection/2d.cpp) --------
class AdvectionAmrOracle:
    """tests/advection/2d.cpp:170-390 on the CPU: initialize.hpp, the
    pre-refinement loop (:260-290), then per step the solver (solve.hpp via
    oracle.dccrg_oracle.AdvectionLists), check_for_adaptation on the
    pre-apply densities, apply_fluxes and adapt_grid (adapter.hpp:184-319),
    every rank simulated.  Geometry: start 0, level-0 cell length 1 / cells
    along every axis (2d.cpp:238-243)."""

    def __init__(self, cells: int, max_ref_lvl: int, comm_size: int = 1, relative_diff=0.025,
                 diff_threshold=0.25, unrefine_sensitivity=0.5, cfl=0.5):
        from oracle.dccrg_oracle import AdvectionLists  # noqa: F401
        self.o = AmrOracle((cells, cells, 1), max_ref_lvl, (True, True, False), 0, comm_size)
        self.l0 = np.array([1.0 / cells] * 3)
        self.params = (relative_diff, diff_threshold, unrefine_sensitivity)
        self.cfl = cfl
        self.state: Dict[int, List[float]] = {}  # cell -> [rho, flux, vx, vy, vz, lx, ly, lz]
        self._init_state()
        for _ in range(self.o.M):
            sets = self.check_for_adaptation()
            self.adapt(sets)
            self._init_state()
        self.dt = self.max_time_step()

    def _geom(self, c):
        m = self.o.mapping
        idx = np.array(m.get_indices(c), dtype=np.float64)
        ln = self.l0 / 2.0 ** self.o.level(c)
        return idx * (self.l0 / 2.0 ** self.o.M) + ln / 2, ln

    def _init_state(self):
        """initialize.hpp:27-65."""
        self.state = {}
        for c in self.o.cells():
            ctr, ln = self._geom(c)
            r = min(np.sqrt((ctr[0] - 0.25) ** 2 + (ctr[1] - 0.5) ** 2), 0.15) / 0.15
            self.state[c] = [0.25 * (1 + np.cos(np.pi * r)), 0.0, -ctr[1] + 0.5, ctr[0] - 0.5, 0.0,
                             ln[0], ln[1], ln[2]]

    def _lists(self):
        from oracle.dccrg_oracle import AdvectionLists
        return AdvectionLists(self.o.grid, self.o.P)

    def arrays(self):
        """cells ascending, and the state columns rho, flux, vx, vy, vz, lx,
        ly, lz as contiguous arrays (the C restatement takes raw pointers)"""
        cells = self.o.cells()
        a = np.array([self.state[c] for c in cells])
        return cells, [np.ascontiguousarray(a[:, k]) for k in range(8)]

    def max_time_step(self) -> float:
        cells, a = self.arrays()
        lists = self._lists()
        return lists.max_time_step([a[0], a[2], a[3], a[4], a[5], a[6], a[7]])

    def check_for_adaptation(self):
        """adapter.hpp:43-176, per rank, cells visited in ascending order."""
        from oracle.dccrg_oracle import iteration_cache_lists
        o = self.o
        rel, thr, sens = self.params
        inc = rel / o.M
        sets = []
        for r in range(o.P):
            local = [c for c in o.cells() if o.owner(c) == r]
            maxd = {c: 0.0 for c in local}
            for c in local:
                lc = o.mapping.get_cell_length_in_indices(c)
                nof = o.grid.find_neighbors_of(c)
                nto = o.grid.find_neighbors_to(c)
                lof, _ = iteration_cache_lists(nof, nto)
                for n, off in lof:
                    ln = o.mapping.get_cell_length_in_indices(n)
                    x, y, z = off
                    face = ((x == lc or x == -ln) and y == 0 and z == 0) or \
                           ((y == lc or y == -ln) and x == 0 and z == 0) or \
                           ((z == lc or z == -ln) and x == 0 and y == 0)
                    if not face:
                        continue
                    a, b = self.state[c][0], self.state[n][0]
                    diff = abs(a - b) / (min(a, b) + thr)
                    maxd[c] = max(diff, maxd[c])
                    if o.owner(n) == r:
                        maxd[n] = max(diff, maxd[n])
            to_ref, keep, unref = set(), set(), set()
            for c in local:
                lvl = o.level(c)
                refine_diff = (lvl + 1) * inc
                unrefine_diff = sens * refine_diff
                sibs = o.siblings(c)
                diff = maxd[c]
                if diff > refine_diff:
                    to_ref.add(c)
                    for s in sibs:
                        unref.discard(s)
                        keep.discard(s)
                elif diff >= unrefine_diff:
                    dont = not any(s in to_ref or s in keep for s in sibs)
                    if dont and lvl > 0:
                        keep.add(c)
                        for s in sibs:
                            unref.discard(s)
                else:
                    un = not any(s in to_ref or s in keep for s in sibs)
                    if un and lvl > 0:
                        unref.add(c)
            sets.append((sorted(to_ref), sorted(keep), sorted(unref)))
        return sets

    def adapt(self, sets):
        """adapter.hpp:184-319 on every rank, then one stop_refining."""
        o = self.o
        for r, (to_ref, keep, unref) in enumerate(sets):
            for c in to_ref:
                o.refine_completely(r, c)
            for c in keep:
                o.dont_unrefine(r, c)
            for c in unref:
                o.unrefine_completely(r, c)
        old = self.state
        new = o.stop_refining()
        st = {c: old[c] for c in o.cells() if c in old}
        for r in range(o.P):
            for c in new[r]:
                p = o.mapping.get_parent(c)
                st[c] = [old[p][0], 0.0] + [0.0] * 6
            rem = o.get_removed_cells(r)
            parents = sorted(set(o.mapping.get_parent(c) for c in rem))
            for p in parents:
                st[p] = [0.0, 0.0] + [0.0] * 6
            for c in rem:
                st[o.mapping.get_parent(c)][0] += old[c][0] / 8
        for c in o.cells():  # velocities and lengths (:303-313)
            ctr, ln = self._geom(c)
            st[c][2:] = [-ctr[1] + 0.5, ctr[0] - 0.5, 0.0, ln[0], ln[1], ln[2]]
        self.state = st

    def step(self):
        """2d.cpp:321-444 with adapt_n = 1."""
        cells, a = self.arrays()
        sets = self.check_for_adaptation()
        lists = self._lists()
        rho = lists.step([a[0], a[2], a[3], a[4], a[5], a[6], a[7]], self.cfl * self.dt)
        for i, c in enumerate(cells):
            self.state[c][0] = rho[i]
            self.state[c][1] = 0.0
        self.adapt(sets)
        self.dt = self.max_time_step()
