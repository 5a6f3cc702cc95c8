"""GPU parity of the AMR-aware game of life (tests/game_of_life/solve.hpp:
40-170, dccrgx_gol_amr_step) against the oracle's literal restatement
(oracle.dccrg_oracle.GolHierarchical): the 15x15 KAT of game_of_life_test.cpp
on a uniform grid, and refined grids (cells refined once, hood 1) at 1-3
ranks, where the state must also equal the unrefined game (refined2d.cpp's
property).  The whole 9 x u64 cell is compared bit for bit after every step.
"""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from dccrg_amd import _capi as X  # noqa: E402
from oracle import dccrg_oracle as O  # noqa: E402

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
DEV = torch.device("cuda", 0)
CELL = np.dtype((np.uint64, 9))


def grids_for(length, M, periodic, hood, leaves, P):
    out = []
    for r in range(P):
        c = D.Context(0, r, P)
        g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*periodic)
             .set_neighborhood_length(hood).initialize(c, leaves=leaves))
        g._keep = c
        g.add_field("data", CELL)
        out.append(g)
    return out


def loopback_halo(grids):
    """update_copies_of_remote_neighbors on every rank, messages moved
    through device buffers (one process emulates the ranks)."""
    msgs = {}
    for r, g in enumerate(grids):
        for p in g.get_cells_to_send():
            buf = torch.empty(1 << 22, dtype=torch.uint8, device=DEV)
            torch.cuda.synchronize()
            msgs[(r, p)] = (buf, g.pack_to(p, buf.data_ptr(), buf.numel(), fields=["data"]))
            g.ctx.synchronize()
    for r, g in enumerate(grids):
        g.halo_self(fields=["data"])
        for p in g.get_cells_to_receive():
            buf, n = msgs[(p, r)]
            g.unpack_from(p, buf.data_ptr(), n, fields=["data"])
        g.ctx.synchronize()


def step(grids):
    """game_of_life_test.cpp:378-414: update, then get_live_neighbors."""
    if len(grids) == 1:
        grids[0].update_copies_of_remote_neighbors(fields=["data"])
        grids[0].gol_amr_step("data")
        return
    loopback_halo(grids)
    for g in grids:
        g.gol_amr_phase("data", X.GOLH_RECORD)
    loopback_halo(grids)
    for g in grids:
        g.gol_amr_phase("data", X.GOLH_SPREAD_APPLY)


def state(grids):
    ids = np.concatenate([g.local_cells() for g in grids])
    data = np.concatenate([g.read_local("data") for g in grids])
    order = np.argsort(ids)
    return ids[order], data[order]


def oracle_state(s):
    return np.array(s.cells, dtype=np.uint64), np.array([s.data[c] for c in s.cells], dtype=np.uint64)


def test_kat_15x15_uniform():
    k = GOLD["gol_kat"]
    g = grids_for(k["length"], 0, k["periodic"], k["hood_length"], None, 1)
    s = O.GolHierarchical(O.Grid(k["length"], 0, k["periodic"], k["hood_length"]))
    n = int(np.prod(k["length"]))
    d = np.zeros((n, 9), dtype=np.uint64)
    d[np.array(k["initial_live"]) - 1, 0] = 1
    g[0].write_local("data", d)
    for c in k["initial_live"]:
        s.data[c][0] = 1
    for t in range(k["steps"]):
        ids, got = state(g)
        live = set(ids[got[:, 0] != 0].tolist())
        assert set(k["always_alive"]) <= live, t
        assert set(k["alive_even_steps" if t % 2 == 0 else "alive_odd_steps"]) <= live, t
        if str(t) in k["glider"]:
            assert set(k["glider"][str(t)]) <= live, t
        assert np.array_equal(got, oracle_state(s)[1]), t
        step(g)
        s.halo()
        s.get_live_neighbors()


def refined_leaves(length, n_refine, seed):
    rng = np.random.default_rng(seed)
    m = O.Mapping(length, 1)
    n0 = int(np.prod(length))
    refined = set(int(v) for v in rng.choice(np.arange(1, n0 + 1), size=n_refine, replace=False))
    leaves = []
    for c in range(1, n0 + 1):
        leaves += m.get_all_children(c) if c in refined else [c]
    return sorted(leaves)


@pytest.mark.parametrize("length,periodic,n_refine,P", [
    ((12, 10, 1), (True, True, False), 30, 1),
    ((16, 16, 1), (True, True, False), 100, 1),
    ((9, 9, 1), (False, False, False), 20, 3),
    ((8, 11, 1), (True, False, False), 40, 2),
    ((10, 6, 1), (True, True, False), 25, 3),
])
def test_refined_matches_oracle_and_unrefined_game(length, periodic, n_refine, P):
    leaves = refined_leaves(length, n_refine, 11)
    grids = grids_for(length, 1, periodic, 1, leaves, P)
    og = O.Grid(length, 1, periodic, 1, leaves=leaves)
    s = O.GolHierarchical(og, P)
    n0 = int(np.prod(length))
    alive0 = O.random_alive(np.arange(1, n0 + 1, dtype=np.uint64), 300)
    for c in s.cells:
        s.data[c][0] = int(alive0[s.par[c] - 1])
    for g in grids:
        loc = g.local_cells()
        d = np.zeros((loc.size, 9), dtype=np.uint64)
        d[:, 0] = [s.data[int(c)][0] for c in loc]
        g.write_local("data", d)
    steps = 8
    for t in range(steps):
        ids, got = state(grids)
        assert ids.tolist() == s.cells
        assert np.array_equal(got, oracle_state(s)[1]), t
        want, _ = O.gol_reference_run(length, periodic, 1, alive0.astype(np.uint32), t)
        assert np.array_equal(got[:, 0], want[np.array([s.par[c] - 1 for c in s.cells])]), t
        step(grids)
        s.halo()
        s.get_live_neighbors()
    for g in grids:
        g.close()


def test_errors_match_reference_aborts():
    # more than 8 live level-0 parents (3-D, everything alive): solve.hpp:93-96
    g = grids_for((4, 4, 4), 0, (True, True, True), 1, None, 1)[0]
    g.write_local("data", np.ones((64, 9), dtype=np.uint64) * np.array([1] + [0] * 8, dtype=np.uint64))
    with pytest.raises(D.DccrgxError) as e:
        g.gol_amr_step("data")
    assert e.value.code == 5
    # wrong element size
    g.add_field("small", np.uint32)
    with pytest.raises(D.DccrgxError):
        g.gol_amr_step("small")
    g.close()
