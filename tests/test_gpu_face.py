"""GPU parity of get_face_neighbors_of (dccrg.hpp:2828-2955) over the face
graph (update_neighbors_, :9463-9597): the reference tests' known answers
(tests/get_face_neighbors/test1.cpp) on the device, and the oracle's
restatement on uniform and mixed-refinement grids."""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from oracle import dccrg_oracle as O  # noqa: E402
from test_gpu_explicit import CASES, leaves_for  # noqa: E402

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))


def refined(length, M, refine):
    m = O.Mapping(length, M)
    cells = set(range(1, int(np.prod(length)) + 1))
    for c in refine:
        cells.discard(c)
        cells |= set(m.get_all_children(c))
    return sorted(cells)


def grid(length, M, per, hood, leaves):
    c = D.Context(0, 0, 1)
    g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
         .set_neighborhood_length(hood).initialize(c, leaves=leaves))
    g._keep = c
    return g


@pytest.mark.parametrize("case", GOLD["face_neighbor_counts"], ids=lambda c: c["src"])
def test_face_neighbor_kats_on_device(case):
    length, M = tuple(case["length"]), case["max_ref_lvl"]
    leaves = refined(length, M, case["refine"]) if case["refine"] else None
    g = grid(length, M, tuple(bool(p) for p in case["periodic"]), 1, leaves)
    cells = np.array(leaves if leaves else range(1, int(np.prod(length)) + 1), dtype=np.uint64)
    row, ids, dirs = g.face_neighbors_of(cells)
    for i, c in enumerate(cells):
        got = [int(v) for v in ids[int(row[i]):int(row[i + 1])]]
        assert len(got) == case["count"], (case["src"], int(c))
        if "ids" in case:
            assert got == case["ids"][str(int(c))]


@pytest.mark.parametrize("case", CASES)
def test_face_neighbors_explicit(case):
    leaves = leaves_for(case)
    length, M, per, hood = case[:4]
    og = O.Grid(length, M, per, hood, leaves)
    g = grid(length, M, per, hood, leaves)
    row, ids, dirs = g.face_neighbors_of(np.array(leaves, dtype=np.uint64))
    for i, c in enumerate(leaves):
        got = [(int(ids[k]), int(dirs[k])) for k in range(int(row[i]), int(row[i + 1]))]
        assert got == og.face_neighbors_of(c), c


@pytest.mark.parametrize("length,per", [((5, 4, 3), (False, False, False)), ((1, 6, 2), (True, True, False)),
                                        ((7, 1, 1), (True, False, True)), ((3, 3, 3), (True, True, True))])
def test_face_neighbors_uniform(length, per):
    og = O.Grid(length, 2, per, 1)
    g = grid(length, 2, per, 1, None)
    cells = np.arange(1, int(np.prod(length)) + 1, dtype=np.uint64)
    row, ids, dirs = g.face_neighbors_of(cells)
    for i, c in enumerate(cells):
        got = [(int(ids[k]), int(dirs[k])) for k in range(int(row[i]), int(row[i + 1]))]
        assert got == og.face_neighbors_of(int(c))


def test_face_neighbors_missing_cell_fails_loudly():
    g = grid((3, 3, 1), 1, (False, False, False), 1, refined((3, 3, 1), 1, [5]))
    with pytest.raises(D.DccrgxError):
        g.face_neighbors_of(np.array([5], dtype=np.uint64))  # refined: not a leaf
