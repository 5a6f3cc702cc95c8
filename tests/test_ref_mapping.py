"""Mapping and Cartesian geometry against vectors written by the REFERENCE's
own classes (tests/golden/ref_mapping.npz, made by
tests/golden/make_ref_mapping.py from dccrg_mapping.hpp and
dccrg_cartesian_geometry.hpp built where they lie, oracle/Makefile `ref`).

CPU tests pin the oracle restatement and the library's host mapping entry
points; the GPU tests run the batched device kernels over the same ids.
Everything is bit-exact (the geometry too: its divisions are by powers of 2).
"""
import json
import os

import numpy as np
import pytest

from oracle import dccrg_oracle as O

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_mapping.npz"))
META = json.loads(str(GOLD["meta"]))
CASES = META["cases"]
ERROR_CELL = 0
IDS = [c["name"] for c in CASES]


def case(name):
    c = next(c for c in CASES if c["name"] == name)
    return (c, GOLD[name + ".ids"], GOLD[name + ".rec"], GOLD[name + ".geo"], GOLD[name + ".q"],
            GOLD[name + ".qcell"])


def valid(c, rec):
    lvl = rec[:, 3].view(np.int64)
    return (lvl >= 0) & (lvl <= c["max_ref_lvl"])


def test_fixture_covers_survey_grids():
    names = set(IDS)
    for n in ("c1_10x10x1_l0", "t_3x3x1_l1", "c3_400x400x1_l2", "t_100x200x300_l13", "c4_2048c_l0",
              "c4_2048c_l10"):
        assert n in names
    c = next(c for c in CASES if c["name"] == "t_100x200x300_l13")
    assert c["max_possible"] == 13


@pytest.mark.parametrize("name", IDS)
def test_oracle_mapping_matches_reference(name):
    c, ids, rec, geo, q, qcell = case(name)
    m = O.Mapping(c["length"], c["max_ref_lvl"])
    assert m.last_cell == c["last_cell"]
    assert O.max_possible_refinement_level(c["length"]) == c["max_possible"]
    idx, lvl = m.ids_to_indices(ids)
    np.testing.assert_array_equal(idx, rec[:, 0:3])
    np.testing.assert_array_equal(lvl.astype(np.int64), rec[:, 3].view(np.int64))
    for i, cell in enumerate(ids.tolist()):
        r = rec[i].tolist()
        assert m.get_indices(cell) == tuple(r[0:3]), cell
        assert m.get_cell_length_in_indices(cell) == r[4], cell
        assert m.get_parent(cell) == r[5], cell
        assert m.get_level_0_parent(cell) == r[6], cell
        assert m.get_child(cell) == r[7], cell
        assert m.get_all_children(cell) == r[8:16], cell
        assert m.get_siblings(cell) == r[16:24], cell
    lv = rec[:, 3].view(np.int64)
    ok = valid(c, rec)
    np.testing.assert_array_equal(m.indices_to_ids(rec[ok, 0:3], lv[ok].astype(np.int32)), rec[ok, 24])
    got = [m.get_cell_from_indices(q[i, :3], int(q[i, 3].view(np.int64))) for i in range(q.shape[0])]
    np.testing.assert_array_equal(np.array(got, dtype=np.uint64), qcell)


@pytest.mark.parametrize("name", IDS)
def test_oracle_geometry_matches_reference(name):
    """The oracle's centre / length formula (advection_initial_state,
    tests/advection/initialize.hpp over get_center / get_length) equals the
    reference Cartesian_Geometry bit for bit; invalid ids give NaN there."""
    c, ids, rec, geo, q, qcell = case(name)
    ok = valid(c, rec) & (ids != 0)
    assert np.isnan(geo[~ok]).all()
    lvl = rec[ok, 3].view(np.int64)
    l0 = np.array(c["level_0_cell_length"])
    start = np.array(c["start"])
    M = c["max_ref_lvl"]
    length = l0[None, :] * (1.0 / (2.0 ** lvl.astype(np.float64)))[:, None]
    center = start[None, :] + rec[ok, 0:3].astype(np.float64) * (l0 / float(2 ** M))[None, :] + length / 2
    np.testing.assert_array_equal(length, geo[ok, 0:3])
    np.testing.assert_array_equal(center, geo[ok, 3:6])
    np.testing.assert_array_equal(center - length / 2, geo[ok, 6:9])
    np.testing.assert_array_equal(center + length / 2, geo[ok, 9:12])
    if np.all(start == 0):
        m = O.Mapping(c["length"], M)
        st = O.advection_initial_state(m, ids[ok], l0)
        np.testing.assert_array_equal(np.stack(st[4:7], 1), geo[ok, 0:3])
        np.testing.assert_array_equal(-geo[ok, 4] + 0.5, st[1])
        np.testing.assert_array_equal(geo[ok, 3] - 0.5, st[2])


@pytest.mark.parametrize("name", IDS)
def test_library_host_mapping_matches_reference(name):
    """The library's host entry points (dccrgx_map_host_*; no device)."""
    import dccrg_amd as D
    from dccrg_amd import _capi as X
    c, ids, rec, geo, q, qcell = case(name)
    m = D.Mapping(c["length"], c["max_ref_lvl_arg"])
    assert m.max_ref_lvl == c["max_ref_lvl"]
    assert m.get_last_cell() == c["last_cell"]
    idx, lvl = m.levels_and_indices(ids)
    np.testing.assert_array_equal(idx, rec[:, 0:3])
    np.testing.assert_array_equal(lvl.astype(np.int64), rec[:, 3].view(np.int64))
    for col, op in ((4, X.OP_LENGTH_IN_INDICES), (5, X.OP_PARENT), (6, X.OP_LEVEL_0_PARENT), (7, X.OP_CHILD)):
        np.testing.assert_array_equal(m.ids_op_host(op, ids), rec[:, col], err_msg=str(col))
    for i, cell in enumerate(ids.tolist()):
        assert list(m.get_all_children(cell)) == rec[i, 8:16].tolist(), cell
        assert list(m.get_siblings(cell)) == rec[i, 16:24].tolist(), cell
    got = [m.get_cell_from_indices(q[i, :3], int(q[i, 3].view(np.int64))) for i in range(q.shape[0])]
    np.testing.assert_array_equal(np.array(got, dtype=np.uint64), qcell)


@pytest.mark.gpu
@pytest.mark.parametrize("name", IDS)
def test_device_mapping_matches_reference(name):
    torch = pytest.importorskip("torch")
    import dccrg_amd as D
    from dccrg_amd import _capi as X
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    dev = torch.device("cuda", 0)
    c, ids, rec, geo, q, qcell = case(name)
    m = D.Mapping(c["length"], c["max_ref_lvl_arg"])
    t = torch.from_numpy(ids.view(np.int64).copy()).to(dev)
    idx, lvl = m.ids_to_indices(t)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint64), rec[:, 0:3])
    np.testing.assert_array_equal(lvl.cpu().numpy().astype(np.int64), rec[:, 3].view(np.int64))
    for col, op in ((4, X.OP_LENGTH_IN_INDICES), (5, X.OP_PARENT), (6, X.OP_LEVEL_0_PARENT), (7, X.OP_CHILD)):
        out = m.ids_op(op, t)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), rec[:, col], err_msg=str(col))
    qi = torch.from_numpy(q[:, :3].view(np.int64).copy()).to(dev)
    ql = torch.from_numpy(q[:, 3].view(np.int64).astype(np.int32)).to(dev)
    cells = m.indices_to_ids(qi, ql)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(cells.cpu().numpy().view(np.uint64), qcell)
