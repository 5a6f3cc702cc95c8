"""Variable-size cell data on the device (tests/variable_data_size): per-cell
element counts, receiver-sized ghosts, halo messages with each cell's
elements in ascending id order, mixed with fixed-size fields; uniform and
mixed-level grids, 1-3 ranks (loopback transport)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from test_gpu_explicit import leaves_for, loopback  # noqa: E402
from test_gpu_parity import loopback_halo  # noqa: E402


def grids_for(length, per, hood, P, M=0, leaves=None):
    out = []
    for r in range(P):
        c = D.Context(0, r, P)
        g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
             .set_neighborhood_length(hood).initialize(c, leaves=leaves))
        g._keep = c
        out.append(g)
    return out


def exchange(grids, fields, uniform):
    if len(grids) == 1:
        grids[0].update_copies_of_remote_neighbors(fields=fields)
    elif uniform:
        loopback_halo(grids, fields)
    else:
        loopback(grids, fields)


@pytest.mark.parametrize("P", [1, 2, 3])
def test_variable_neighbour_data_kat(P):
    """variable_neighbour_data.cpp:82-130: 3x1x1, hood 1, cell c holds
    variables1 = [c, c+1, ..] and variables2 = [-c, -(c+1), ..] (c values);
    ghosts are sized by the receiver, then one update moves both."""
    grids = grids_for((3, 1, 1), (False, False, False), 1, P)
    for g in grids:
        g.add_variable_field("v1", np.int32)
        g.add_variable_field("v2", np.int32)
        local = [int(c) for c in g.local_cells()]
        g.resize("v1", local, local)
        g.resize("v2", local, local)
        g.write_cells("v1", local, [np.arange(c, 2 * c) for c in local])
        g.write_cells("v2", local, [-np.arange(c, 2 * c) for c in local])
        remote = [int(c) for c in g.remote_cells()]
        g.resize("v1", remote, remote)
        g.resize("v2", remote, remote)
    exchange(grids, ["v1", "v2"], True)
    seen = {}
    for g in grids:
        for c in (int(x) for x in g.local_cells()):
            assert g.read_cells("v1", [c])[0].tolist() == list(range(c, 2 * c))
            nbrs = [n for n, _ in g.get_neighbors_of(c)]
            got = g.read_cells("v2", nbrs)
            seen[c] = [v for arr in got for v in arr.tolist()]
    # cell 1's neighbor is 2, cell 2's are 1 and 3, cell 3's is 2
    assert seen == {1: [-2, -3], 2: [-1, -3, -4, -5], 3: [-2, -3]}


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("per", [(False, False, True), (True, True, False)])
def test_variable_uniform_mixed_message(P, per):
    """Random counts 0..5 of f64 plus a fixed u32 field in the same message."""
    length = (6, 5, 9)
    grids = grids_for(length, per, 1, P)
    rng = np.random.default_rng(P)
    n = int(np.prod(length))
    counts = rng.integers(0, 6, n + 1)
    payload = {c: rng.standard_normal(counts[c]) for c in range(1, n + 1)}
    for g in grids:
        g.add_variable_field("var", np.float64)
        g.add_field("tag", np.uint32)
        local = [int(c) for c in g.local_cells()]
        g.resize("var", local, counts[local])
        g.write_cells("var", local, [payload[c] for c in local])
        g.write_local("tag", np.array(local, dtype=np.uint32) * 7)
        remote = [int(c) for c in g.remote_cells()]
        if remote:
            g.resize("var", remote, counts[remote])
    exchange(grids, ["var", "tag"], True)
    for g in grids:
        remote = [int(c) for c in g.remote_cells()]
        recv = set(c for v in g.get_cells_to_receive().values() for c in v)
        for c, arr in zip(remote, g.read_cells("var", remote)):
            if c in recv:
                assert np.array_equal(arr, payload[c]), c
        for c, t in zip(remote, g.read_remote("tag")):
            if c in recv:
                assert int(t) == 7 * c


@pytest.mark.parametrize("case_i", [2, 5, 8])
def test_variable_mixed_level(case_i):
    from test_gpu_explicit import CASES
    case = CASES[case_i]
    leaves = leaves_for(case)
    length, M, per, hood = case[:4]
    P = 3
    grids = grids_for(length, per, hood, P, M, leaves)
    cnt = {c: (c % 4) for c in leaves}
    for g in grids:
        g.add_variable_field("var", np.int64)
        local = [int(c) for c in g.local_cells()]
        g.resize("var", local, [cnt[c] for c in local])
        g.write_cells("var", local, [np.full(cnt[c], c, dtype=np.int64) for c in local])
        remote = [int(c) for c in g.remote_cells()]
        if remote:
            g.resize("var", remote, [cnt[c] for c in remote])
    exchange(grids, ["var"], False)
    for g in grids:
        recv = set(c for v in g.get_cells_to_receive().values() for c in v)
        remote = [int(c) for c in g.remote_cells()]
        for c, arr in zip(remote, g.read_cells("var", remote)):
            if c in recv:
                assert arr.tolist() == [c] * cnt[c]


def test_resize_keeps_prefix_and_zero_fills():
    g = grids_for((4, 4, 1), (False, False, False), 1, 1)[0]
    g.add_variable_field("v", np.float32)
    cells = [int(c) for c in g.local_cells()]
    g.resize("v", cells, 3)
    g.write_cells("v", cells, [np.array([c, c + 0.5, c + 0.25], dtype=np.float32) for c in cells])
    g.resize("v", cells[:5], 5)
    g.resize("v", cells[5:], 1)
    for c, arr in zip(cells, g.read_cells("v", cells)):
        if c in cells[:5]:
            assert arr.tolist() == [c, c + 0.5, c + 0.25, 0.0, 0.0]
        else:
            assert arr.tolist() == [c]
    with pytest.raises(D.DccrgxError):
        g.write_local("v", np.zeros(16, dtype=np.float32))  # fixed-size API refuses


def test_fixed_field_cell_access():
    """operator[] style access by id for a fixed-size field, ghosts included."""
    grids = grids_for((5, 4, 6), (False, False, True), 1, 2)
    for g in grids:
        g.add_field("x", np.float64)
        local = [int(c) for c in g.local_cells()]
        g.write_cells("x", local, np.array(local, dtype=np.float64) / 3)
    loopback_halo(grids, ["x"])
    for g in grids:
        remote = [int(c) for c in g.remote_cells()]
        vals = np.concatenate(g.read_cells("x", remote))
        assert np.array_equal(vals, np.array(remote, dtype=np.float64) / 3)
        local = [int(c) for c in g.local_cells()]
        assert np.array_equal(np.concatenate(g.read_cells("x", local)), g.read_local("x"))


@pytest.mark.parametrize("P", [1, 2, 3])
def test_variable_counts_change_between_exchanges(P):
    """The pack / unpack / self-copy segments are cached per count epoch
    (halo.hip VarPlan): after every resize (new counts, new values) the next
    exchange must use the new layout.  Fields of 1-, 4- and 8-byte elements
    share each message, so segments start at every alignment."""
    length, per = (5, 4, 6), (True, False, True)
    grids = grids_for(length, per, 1, P)
    n = int(np.prod(length))
    kinds = {"b": np.uint8, "i": np.int32, "d": np.float64}
    for g in grids:
        for name, dt in kinds.items():
            g.add_variable_field(name, dt)
    for rnd in range(3):
        rng = np.random.default_rng(10 * P + rnd)
        counts = {name: rng.integers(0, 7, n + 1) for name in kinds}
        vals = {name: {c: (rng.integers(0, 100, counts[name][c]) + c).astype(dt) for c in range(1, n + 1)}
                for name, dt in kinds.items()}
        for g in grids:
            local = [int(c) for c in g.local_cells()]
            remote = [int(c) for c in g.remote_cells()]
            for name in kinds:
                g.resize(name, local, counts[name][local])
                g.write_cells(name, local, [vals[name][c] for c in local])
                if remote:
                    g.resize(name, remote, counts[name][remote])
        exchange(grids, list(kinds), True)
        for g in grids:
            recv = set(c for v in g.get_cells_to_receive().values() for c in v)
            remote = [int(c) for c in g.remote_cells()]
            for name in kinds:
                for c, arr in zip(remote, g.read_cells(name, remote)):
                    if c in recv or P == 1:
                        assert np.array_equal(arr, vals[name][c]), (rnd, name, c)
