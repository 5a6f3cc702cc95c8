"""The oracle's restatement of the AMR-aware game of life
(tests/game_of_life/solve.hpp:40-170) against the reference's own known
answers: the 15x15 KAT of game_of_life_test.cpp (which runs that solver) and
refined.cpp / refined2d.cpp's property that a grid with refined cells behaves
exactly as the unrefined grid ("emulating unrefined behaviour")."""
import json
import os

import numpy as np
import pytest

from oracle import dccrg_oracle as O

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))


def test_hierarchical_gol_kat_15x15():
    k = GOLD["gol_kat"]
    g = O.Grid(k["length"], 0, k["periodic"], k["hood_length"])
    s = O.GolHierarchical(g)
    for c in k["initial_live"]:
        s.data[c][0] = 1
    for step in range(k["steps"]):
        s.halo()
        live = {c for c in s.cells if s.data[c][0]}
        assert set(k["always_alive"]) <= live, step
        assert set(k["alive_even_steps" if step % 2 == 0 else "alive_odd_steps"]) <= live, step
        if str(step) in k["glider"]:
            assert set(k["glider"][str(step)]) <= live, step
        s.get_live_neighbors()


def refined_case(length, periodic, n_refine, seed, comm_size=1):
    """Level-0 grid with `n_refine` random cells refined once; every child
    starts with its parent's state (refined2d.cpp:206-215)."""
    rng = np.random.default_rng(seed)
    m = O.Mapping(length, 1)
    n0 = int(np.prod(length))
    refined = set(int(v) for v in rng.choice(np.arange(1, n0 + 1), size=n_refine, replace=False))
    leaves = []
    for c in range(1, n0 + 1):
        leaves += m.get_all_children(c) if c in refined else [c]
    g = O.Grid(length, 1, periodic, 1, leaves=sorted(leaves))
    alive0 = O.random_alive(np.arange(1, n0 + 1, dtype=np.uint64), 300)
    s = O.GolHierarchical(g, comm_size)
    for c in s.cells:
        s.data[c][0] = int(alive0[s.par[c] - 1])
    return s, alive0


@pytest.mark.parametrize("length,periodic,n_refine,P", [
    ((12, 10, 1), (True, True, False), 30, 1),
    ((9, 9, 1), (False, False, False), 20, 3),
    ((8, 11, 1), (True, False, False), 40, 2),
])
def test_refined_grid_emulates_unrefined(length, periodic, n_refine, P):
    s, alive0 = refined_case(length, periodic, n_refine, 7, P)
    t, _ = refined_case(length, periodic, n_refine, 7, P)
    steps = 8
    ref_alive, _ = O.gol_reference_run(length, periodic, 1, alive0.astype(np.uint32), 0)
    for step in range(steps):
        want, _ = O.gol_reference_run(length, periodic, 1, alive0.astype(np.uint32), step)
        got = s.alive()
        assert np.array_equal(got, want[np.array([s.par[c] - 1 for c in s.cells])].astype(np.uint64)), step
        s.halo()
        s.get_live_neighbors("ascending")
        t.halo()
        t.get_live_neighbors("descending")
        # one refinement level + hood 1: siblings are mutual neighbors, the
        # result does not depend on the reference's hash iteration order
        assert np.array_equal(s.alive(), t.alive()), step


def test_overflow_is_reported():
    """3-D, hood 1, a fully live grid: more than 8 live level-0 parents."""
    g = O.Grid((4, 4, 4), 0, (True, True, True), 1)
    s = O.GolHierarchical(g)
    for c in s.cells:
        s.data[c][0] = 1
    s.halo()
    with pytest.raises(OverflowError):
        s.get_live_neighbors()
