"""CPU checks of the oracle's advection restatement (tests/advection/solve.hpp).

The reference's advection test has no stored outputs, so the restatement is
pinned by properties the reference solver has by construction: every face
flux leaves one cell and enters the other (solve.hpp:224-230), so total mass
sum(density * volume) is conserved on fully periodic grids; and the result
does not depend on the number of processes (each face is solved once per
pair of processes that see it, with the same inputs).  Parity of the device
path against this restatement is in tests/test_gpu_advection.py.
"""
import numpy as np
import pytest

from oracle import dccrg_oracle as O

CASES = [  # length, max_ref_lvl, periodic, hood, refines, seed
    ((8, 8, 1), 0, (True, True, True), 0, 0, 0),
    ((6, 5, 1), 2, (True, True, True), 0, 12, 1),
    ((4, 4, 2), 1, (True, True, True), 1, 10, 2),
    ((5, 4, 1), 2, (False, True, False), 0, 15, 3),
]


def setup(case, P):
    length, M, per, hood, nref, seed = case
    leaves = O.random_balanced_leaves(length, M, per, hood, nref, seed) if nref else None
    g = O.Grid(length, M, per, hood, leaves)
    lists = O.AdvectionLists(g, P)
    state = O.advection_initial_state(g.mapping, lists.cells)
    return g, lists, state


@pytest.mark.parametrize("case", [c for c in CASES if all(c[2])])
def test_mass_conserved_on_periodic_grids(case):
    _, lists, state = setup(case, 1)
    vol = state[4] * state[5] * state[6]
    m0 = float(np.sum(state[0] * vol))
    dt = 0.5 * lists.max_time_step(state)
    for _ in range(10):
        state[0] = lists.step(state, dt)
    assert abs(float(np.sum(state[0] * vol)) - m0) <= 1e-13 * m0
    assert state[0].min() > -1e-12  # upwind at CFL 0.5 stays non-negative


@pytest.mark.parametrize("case", CASES)
def test_process_count_independent(case):
    _, l1, s1 = setup(case, 1)
    _, l3, s3 = setup(case, 3)
    dt = 0.5 * l1.max_time_step(s1)
    assert dt == 0.5 * l3.max_time_step(s3)
    for _ in range(5):
        s1[0] = l1.step(s1, dt)
        s3[0] = l3.step(s3, dt)
    assert np.allclose(s1[0], s3[0], rtol=0, atol=1e-14 * np.abs(s1[0]).max())


def test_max_time_step_uniform():
    """solve.hpp:302-320 on an 8x8 grid: min over cells of length / |v| with
    v = (0.5 - y, x - 0.5, 0); vz = 0 gives inf, which isnormal() skips."""
    _, lists, state = setup(CASES[0], 1)
    lx = 1 / 8
    vmax = 0.5 - 1 / 16  # the outermost cell centers
    assert lists.max_time_step(state) == pytest.approx(lx / vmax, rel=1e-15)
