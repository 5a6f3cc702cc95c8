"""CPU checks of the oracle's Poisson restatement (tests/poisson/poisson_solve.hpp).

Pinned by the reference test's own pass criterion: tests/poisson/poisson3d.cpp
solves -(81/16) sin(x) cos(2y) sin(z/4) on an 8^3 periodic grid with the
middle refined twice and requires the 2-norm of the error against the
analytic solution (refined cells averaged to level 0) to be < 0.35
(poisson3d.cpp:225-236).  Also: independence of the process count.
"""
import math

import numpy as np
import pytest

from oracle import dccrg_oracle as O

L0 = (2 * math.pi / 8, math.pi / 8, 8 * math.pi / 8)  # poisson3d.cpp:127-136


def induce_refines(grid, m, refines):
    """dccrg.hpp:9730-9800: a cell being refined also refines every coarser
    cell in its neighbors_of / neighbors_to (repeated until nothing new)."""
    todo, out = set(refines), set(refines)
    while todo:
        new = set()
        for c in todo:
            lvl = m.get_refinement_level(c)
            for n in [n for n, _ in grid.find_neighbors_of(c)] + grid.find_neighbors_to(c):
                if n and grid.exists(n) and m.get_refinement_level(n) < lvl and n not in out:
                    new.add(n)
        out |= new
        todo = new
    return out


def poisson3d_leaves():
    """poisson3d.cpp:158-178: refine the cells around (pi, pi/2, 4 pi) twice,
    with the reference's induced refines (hood 0).  The survey measured 792
    leaves for this grid."""
    m = O.Mapping((8, 8, 8), 2)
    cells = set(range(1, 513))
    for _ in range(2):
        g = O.Grid((8, 8, 8), 2, (True, True, True), 0, sorted(cells))
        refine = set()
        for c in sorted(cells):
            lo, hi = geometry(m, [c])
            lo, hi = lo[0], hi[0]
            if (lo[0] < 1.01 * math.pi and hi[0] > 0.99 * math.pi and lo[1] < 0.51 * math.pi
                    and hi[1] > 0.49 * math.pi and lo[2] < 4.01 * math.pi and hi[2] > 3.99 * math.pi):
                if m.get_refinement_level(c) < m.max_ref_lvl:
                    refine.add(c)
        for c in induce_refines(g, m, refine):
            cells.discard(c)
            cells |= set(m.get_all_children(c))
    return m, sorted(cells)


def geometry(m, cells):
    """Cartesian_Geometry get_min / get_max with start 0."""
    idx, lvl = m.ids_to_indices(np.asarray(cells, dtype=np.uint64))
    unit = np.array(L0) / 2 ** m.max_ref_lvl
    ln = np.array(L0)[None, :] / (2.0 ** lvl.astype(np.float64))[:, None]
    lo = idx.astype(np.float64) * unit[None, :]
    return lo, lo + ln


def solution_value(x, y, z):
    return np.sin(x) * np.cos(2 * y) * np.sin(z / 4)


def setup(P):
    m, leaves = poisson3d_leaves()
    g = O.Grid((8, 8, 8), 2, (True, True, True), 0, leaves)
    lo, hi = geometry(m, leaves)
    ln = hi - lo
    center = (lo + hi) / 2
    rhs = -(81.0 / 16.0) * solution_value(center[:, 0], center[:, 1], center[:, 2])
    sysm = O.PoissonSystem(g, P, (ln[:, 0], ln[:, 1], ln[:, 2]))
    return m, leaves, sysm, rhs


def error_norm(m, leaves, sol):
    """poisson3d.cpp:61-111: average to level 0, 2-norm vs analytic."""
    avg = {}
    for c, s in zip(leaves, sol):
        p = m.get_level_0_parent(c)
        avg[p] = avg.get(p, 0.0) + s / 8.0 ** m.get_refinement_level(c)
    m0 = O.Mapping((8, 8, 8), 0)
    ids = np.array(sorted(avg), dtype=np.uint64)
    idx, _ = m0.ids_to_indices(ids)
    ctr = (idx.astype(np.float64) + 0.5) * np.array(L0)[None, :]
    exact = solution_value(ctr[:, 0], ctr[:, 1], ctr[:, 2])
    return float(np.sqrt(np.sum((np.array([avg[int(i)] for i in ids]) - exact) ** 2)))


def test_poisson3d_uniform_matches_direct_solve():
    """poisson3d.cpp's problem on the unrefined 8^3 grid: BiCG reaches the
    discrete solution (checked against a dense least-squares solve of the
    operator assembled from the cached factors, :940-971), whose error vs
    the analytic solution is the 7-point stencil's truncation error:
    u_h = u * (81/16) / sum_d (2 - 2 cos(k_d h_d)) / h_d^2."""
    m = O.Mapping((8, 8, 8), 0)
    leaves = list(range(1, 513))
    g = O.Grid((8, 8, 8), 0, (True, True, True), 0, None)
    lo, hi = geometry(m, leaves)
    ln, c = hi - lo, (lo + hi) / 2
    exact = solution_value(c[:, 0], c[:, 1], c[:, 2])
    rhs = -(81.0 / 16.0) * exact
    s = O.PoissonSystem(g, 1, (ln[:, 0], ln[:, 1], ln[:, 2]))
    sol, it, res = s.solve(rhs, np.zeros(512))
    assert res <= 1e-15 and it < 1000
    A = np.zeros((512, 512))
    for k, i in enumerate(s.info):
        A[i, i] = s.sf[i]
        for e in range(int(s.row[k]), int(s.row[k + 1])):
            d = (int(s.code[e]) & 15) - 3
            A[i, s.nb[e]] += s.f[i, 2 * (d - 1) if d > 0 else 2 * (-d - 1) + 1]
    direct = np.linalg.lstsq(A, rhs, rcond=None)[0]
    assert np.abs(sol - direct).max() <= 1e-10
    k = [(1, L0[0]), (2, L0[1]), (0.25, L0[2])]
    lam = sum((2 - 2 * math.cos(kk * h)) / h ** 2 for kk, h in k)
    assert np.allclose(sol, exact * (81.0 / 16.0) / lam, atol=1e-10)
    assert error_norm(m, leaves, sol) == pytest.approx(0.4256, abs=2e-3)


def test_poisson3d_pass_criterion():
    """poisson3d.cpp end to end: the twice-refined grid with induced refines
    has the 792 leaves the survey measured on the reference, and the solution
    meets the reference's own criterion (error 2-norm < 0.35, :225-236).
    The system is non-symmetric: BiCG stops on the residual-increase rule
    and returns the best iterate (:378-404)."""
    m, leaves, sysm, rhs = setup(1)
    assert len(leaves) == 792
    sol, it, res = sysm.solve(rhs, np.zeros(len(leaves)))
    assert 1 <= it <= 1000 and np.isfinite(res)
    assert error_norm(m, leaves, sol) < 0.35


@pytest.mark.parametrize("P", [2, 3])
def test_poisson_process_count_independent(P):
    _, leaves, s1, rhs = setup(1)
    _, _, sP, _ = setup(P)
    a, _, _ = s1.solve(rhs, np.zeros(len(leaves)), max_iterations=20)
    b, _, _ = sP.solve(rhs, np.zeros(len(leaves)), max_iterations=20)
    assert np.abs(a - b).max() <= 1e-12 * np.abs(a).max()


def test_poisson_boundary_and_skip_cells():
    """Cells outside `cells` keep their values (boundary); skipped cells and
    boundary-boundary pairs are dropped (poisson_solve.hpp:892-960)."""
    m = O.Mapping((10, 1, 1), 0)
    g = O.Grid((10, 1, 1), 0, (False, False, False), 0)
    ln = np.full(10, 0.1)
    solve = list(range(3, 9))
    sysm = O.PoissonSystem(g, 1, (ln, ln, ln), solve_cells=solve, skip_cells=[10])
    assert sysm.type[9] == O.POISSON_SKIP and sysm.type[0] == O.POISSON_SKIP  # 1: only boundary nbrs
    x = np.linspace(0.05, 0.95, 10)
    rhs = np.zeros(10)
    guess = np.where(np.isin(np.arange(1, 11), solve), 0.0, x)  # boundary cells hold x
    sol, it, _ = sysm.solve(rhs, guess)
    # 1-D Laplace between fixed boundary values is linear
    assert np.allclose(sol[2:8], x[2:8], atol=1e-10)
    assert np.array_equal(sol[[0, 1, 8, 9]], guess[[0, 1, 8, 9]])
    del m
