"""GPU parity of the advection solver (tests/advection/solve.hpp) against the
oracle's restatement, on uniform and mixed-refinement grids, one and several
processes (loopback halo).  fp64; the device sums a cell's face fluxes in a
different order than the reference's scatter, so densities are compared at
1e-12 * max|density| (per-face fluxes themselves are evaluated identically)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from oracle import dccrg_oracle as O  # noqa: E402
from test_gpu_explicit import leaves_for, loopback  # noqa: E402
from test_gpu_parity import loopback_halo  # noqa: E402

TOL = 1e-12
NAMES = ("density", "vx", "vy", "vz", "length_x", "length_y", "length_z")

CASES = [  # length, max_ref_lvl, periodic, hood, refines, seed  (refines None: uniform)
    ((8, 8, 1), 0, (True, True, True), 0, None, 0),
    ((12, 9, 1), 0, (False, True, False), 0, None, 0),
    ((6, 4, 5), 0, (True, False, True), 1, None, 0),
    ((1, 7, 9), 2, (False, True, True), 0, None, 0),
    ((3, 3, 1), 1, (True, True, False), 0, 10, 2),
    ((6, 5, 1), 2, (True, True, True), 0, 12, 1),
    ((4, 3, 2), 2, (False, False, False), 0, 20, 3),
    ((4, 4, 2), 1, (True, True, True), 1, 10, 2),
    ((3, 4, 3), 1, (True, False, False), 1, 30, 6),
]


def build(case, P):
    length, M, per, hood, nref, seed = case
    leaves = None if nref is None else leaves_for((length, M, per, hood, nref, seed))
    og = O.Grid(length, M, per, hood, leaves)
    lists = O.AdvectionLists(og, P)
    grids = []
    for r in range(P):
        c = D.Context(0, r, P)
        g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
             .set_neighborhood_length(hood).initialize(c, leaves=leaves))
        g._keep = c
        g.add_advection_fields()
        grids.append(g)
    return lists, grids


def exchange(grids, fields, uniform):
    if len(grids) == 1:
        grids[0].update_copies_of_remote_neighbors(fields=list(fields))
        grids[0].ctx.synchronize()
    elif uniform:
        loopback_halo(grids, list(fields))
    else:
        loopback(grids, list(fields))


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("case", CASES)
def test_advection_parity(case, P):
    uniform = case[4] is None
    lists, grids = build(case, P)
    state = O.advection_initial_state(O.Mapping(case[0], case[1]), lists.cells)
    pos = {c: i for i, c in enumerate(lists.cells)}
    idx = []
    for g in grids:
        ix = np.array([pos[int(c)] for c in g.local_cells()], dtype=np.int64)
        idx.append(ix)
        for name, arr in zip(NAMES, state):
            g.write_local(name, arr[ix])
    exchange(grids, NAMES, uniform)  # initialize.hpp:60: everything once
    assert min(g.max_time_step() for g in grids) == lists.max_time_step(state)
    dt = 0.5 * lists.max_time_step(state)
    for _ in range(6):
        state[0] = lists.step(state, dt)
        if P == 1:
            grids[0].advect_step(dt)
        else:
            exchange(grids, ["density"], uniform)
            for g in grids:
                g.calculate_fluxes(dt, True)
                g.calculate_fluxes(dt, False)
                g.apply_fluxes()
    scale = np.abs(state[0]).max()
    for g, ix in zip(grids, idx):
        got = g.read_local("density")
        assert np.abs(got - state[0][ix]).max() <= TOL * scale
        assert np.all(g.read_local("flux") == 0)


@pytest.mark.parametrize("case", CASES)
def test_fused_step_equals_fluxes_then_apply(case):
    """dccrgx_advect_step (one kernel writing the new density into the other
    buffer) against calculate_fluxes(all) + apply_fluxes: bit-identical
    densities, flux 0 afterwards, also when flux starts non-zero; remote
    ghost copies and the buffer swap survive many steps."""
    uniform = case[4] is None
    lists, (a,) = build(case, 1)
    _, (b,) = build(case, 1)
    state = O.advection_initial_state(O.Mapping(case[0], case[1]), lists.cells)
    rng = np.random.default_rng(7)
    flux0 = rng.standard_normal(len(lists.cells)) * 1e-3
    for g in (a, b):
        for name, arr in zip(NAMES, state):
            g.write_local(name, arr)
        g.write_local("flux", flux0)
        exchange([g], NAMES, uniform)
    dt = 0.5 * lists.max_time_step(state)
    for k in range(7):
        a.advect_step(dt)
        b.update_copies_of_remote_neighbors(fields=["density"])
        b.calculate_fluxes(dt, True, region=D._capi.REGION_ALL)
        b.apply_fluxes()
        da, db = a.read_local("density"), b.read_local("density")
        assert np.array_equal(da, db), k
        assert np.all(a.read_local("flux") == 0)
        assert np.array_equal(a.read_remote("density"), b.read_remote("density"))
    for g in (a, b):
        g.close()


def test_advection_mass_conserved_large():
    """Size-independent property at a larger size: 256 x 256 periodic, 20
    steps, total mass conserved to 1e-12 relative."""
    c = D.Context(0, 0, 1)
    n = 256
    g = (D.Dccrg().set_initial_length((n, n, 1)).set_periodic(True, True, True)
         .set_neighborhood_length(0).initialize(c))
    g.add_advection_fields()
    m = O.Mapping((n, n, 1), 0)
    state = O.advection_initial_state(m, g.local_cells())
    for name, arr in zip(NAMES, state):
        g.write_local(name, arr)
    g.update_copies_of_remote_neighbors(fields=list(NAMES))
    vol = state[4] * state[5] * state[6]
    m0 = float(np.sum(state[0] * vol))
    dt = 0.5 * g.max_time_step()
    for _ in range(20):
        g.advect_step(dt)
    rho = g.read_local("density")
    assert abs(float(np.sum(rho * vol)) - m0) <= 1e-12 * m0
    assert rho.min() > -1e-12
    g.close()
    c.close()
