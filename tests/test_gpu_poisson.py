"""GPU parity of the Poisson solver (tests/poisson/poisson_solve.hpp) against
the oracle's restatement: the cached geometric factors bit-exact (same
operation order), BiCG iterates at fixed iteration counts within 1e-12 of
max|x| (fp64; only the dot products' summation order differs), and full
solves to the same converged solution."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from oracle import dccrg_oracle as O  # noqa: E402
from test_oracle_poisson import L0, error_norm, poisson3d_leaves, solution_value  # noqa: E402

TOL = 1e-12


@pytest.fixture(params=["solo", "solo_global", "multi", "rccl"])
def path(request, monkeypatch, lib_options):
    """Every iteration driver: one workgroup for small single-rank systems
    (LDS-resident up to 1024 cells with the 2-norm, else over global memory),
    the batched multi-kernel path used across ranks, and that path through a
    real RCCL communicator (ncclAllReduce of every scalar, periodic images
    as RCCL messages to the rank itself)."""
    monkeypatch.delenv("DCCRGX_TEST_RCCL", raising=False)
    if request.param == "solo_global":
        lib_options("poisson_solo_global", 1)
    elif request.param == "multi":
        lib_options("poisson_multi", 1)
    elif request.param == "rccl":
        monkeypatch.setenv("DCCRGX_TEST_RCCL", "1")
    return request.param


def make_context():
    c = D.Context(0, 0, 1)
    if os.environ.get("DCCRGX_TEST_RCCL"):
        c.comm_init(D.Context.unique_id())
        c.route_self_through_rccl(True)
    return c


def geometry(length, M, cells, l0):
    m = O.Mapping(length, M)
    idx, lvl = m.ids_to_indices(np.asarray(cells, dtype=np.uint64))
    unit = np.array(l0) / 2 ** M
    ln = np.array(l0)[None, :] / (2.0 ** lvl.astype(np.float64))[:, None]
    lo = idx.astype(np.float64) * unit[None, :]
    return ln, lo + ln / 2


CASES = {
    # name: (length, M, periodic, leaves, l0, solve_cells, skip_cells)
    "uniform8": ((8, 8, 8), 0, (True, True, True), None, L0, None, ()),
    "refined792": ((8, 8, 8), 2, (True, True, True), "poisson3d", L0, None, ()),
    "line_boundary": ((10, 1, 1), 0, (False, False, False), None, (0.1, 0.1, 0.1), list(range(3, 9)), [10]),
    "plane_open": ((12, 9, 1), 0, (False, False, False), None, (0.5, 0.25, 1.0), None, ()),
    "stretch_z": ((3, 4, 6), 1, (True, False, True), "random", (1.0, 2.0, 0.5), None, ()),
}


def build(name):
    length, M, per, leaves, l0, solve, skip = CASES[name]
    if leaves == "poisson3d":
        _, leaves = poisson3d_leaves()
    elif leaves == "random":
        leaves = O.random_balanced_leaves(length, M, per, 0, 12, 5)
    og = O.Grid(length, M, per, 0, leaves)
    cells = [int(c) for c in og.cells()]
    ln, ctr = geometry(length, M, cells, l0)
    if name in ("uniform8", "refined792"):
        rhs = -(81.0 / 16.0) * solution_value(ctr[:, 0], ctr[:, 1], ctr[:, 2])
        guess = np.zeros(len(cells))
    else:
        rhs = np.sin(3 * ctr[:, 0]) * np.cos(ctr[:, 1]) + 0.1 * ctr[:, 2]
        guess = ctr[:, 0] * 0.3 - ctr[:, 1] * 0.1
    sysm = O.PoissonSystem(og, 1, (ln[:, 0], ln[:, 1], ln[:, 2]), solve_cells=solve, skip_cells=skip)
    c = make_context()
    g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
         .set_neighborhood_length(0).initialize(c, leaves=leaves))
    g._keep = c
    for f in ("rhs", "solution", "length_x", "length_y", "length_z"):
        g.add_field(f, np.float64)
    assert [int(x) for x in g.local_cells()] == cells
    g.write_local("rhs", rhs)
    g.write_local("length_x", ln[:, 0])
    g.write_local("length_y", ln[:, 1])
    g.write_local("length_z", ln[:, 2])
    return g, sysm, cells, rhs, guess, (solve if solve is not None else cells), skip


@pytest.mark.parametrize("name", sorted(CASES))
def test_poisson_factors_bit_exact(name):
    g, sysm, cells, rhs, guess, solve, skip = build(name)
    s = D.PoissonSolve(g, max_iterations=1)
    g.write_local("solution", guess)
    s.solve(solve, skip)
    assert np.array_equal(g.read_local("poisson.type"), sysm.type)
    info = np.zeros(len(cells), dtype=bool)
    info[sysm.info] = True
    assert np.array_equal(g.read_local("poisson.scaling_factor")[info], sysm.sf[info])
    for k, m in enumerate(("f_x_pos", "f_x_neg", "f_y_pos", "f_y_neg", "f_z_pos", "f_z_neg")):
        assert np.array_equal(g.read_local("poisson." + m)[info], sysm.f[info, k]), m


@pytest.mark.parametrize("iters", [1, 2, 5, 12])
@pytest.mark.parametrize("name", sorted(CASES))
def test_poisson_fixed_iterations(name, iters, path):
    g, sysm, cells, rhs, guess, solve, skip = build(name)
    s = D.PoissonSolve(g, max_iterations=iters)
    g.write_local("solution", guess)
    it, res = s.solve(solve, skip)
    ref, rit, rres = sysm.solve(rhs, guess, max_iterations=iters)
    assert it == rit
    assert res == pytest.approx(rres, rel=1e-9)
    got = g.read_local("solution")
    assert np.abs(got - ref).max() <= TOL * max(np.abs(ref).max(), 1.0)


@pytest.mark.parametrize("name", sorted(CASES))
def test_poisson_full_solve(name, path):
    g, sysm, cells, rhs, guess, solve, skip = build(name)
    s = D.PoissonSolve(g)
    g.write_local("solution", guess)
    it, res = s.solve(solve, skip)
    ref, rit, rres = sysm.solve(rhs, guess)
    got = g.read_local("solution")
    scale = max(np.abs(ref).max(), 1.0)
    # the north-star gate: the oracle's iteration count and stopping rule
    # (converged below stop_residual, or stopped on the residual-increase
    # rule with the same best iterate), and the solution within 1e-12 of
    # max|x|.  Only the dot products' summation order differs (block tree vs
    # the reference's sequential loop), measured at <= 3e-15 of max|x| on
    # every case and iteration driver (tools/poisson_full_diff.py,
    # profiles/r3a_poisson_diff.log)
    assert it == rit
    assert (res <= 1e-15) == (rres <= 1e-15)
    if rres > 1e-15:
        assert res == pytest.approx(rres, rel=1e-9)
    assert np.abs(got - ref).max() <= TOL * scale


def test_poisson_cache_reuse(path):
    """cache_is_up_to_date = true skips cache_system_info (:263-265)."""
    g, sysm, cells, rhs, guess, solve, skip = build("plane_open")
    s = D.PoissonSolve(g, max_iterations=3)
    g.write_local("solution", guess)
    s.solve(solve, skip)
    g.write_local("solution", guess)
    it, _ = s.solve(solve, skip, cache_is_up_to_date=True)
    ref, rit, _ = sysm.solve(rhs, guess, max_iterations=3)
    assert it == rit
    assert np.abs(g.read_local("solution") - ref).max() <= TOL * max(np.abs(ref).max(), 1.0)


def test_poisson3d_reference_criterion_on_device():
    """tests/poisson/poisson3d.cpp end to end on the device: 792 leaves, error
    2-norm vs the analytic solution below the reference's 0.35 (:225-236)."""
    g, sysm, cells, rhs, guess, solve, skip = build("refined792")
    assert len(cells) == 792
    s = D.PoissonSolve(g)
    g.write_local("solution", guess)
    s.solve(solve, skip)
    assert error_norm(O.Mapping((8, 8, 8), 2), cells, g.read_local("solution")) < 0.35
