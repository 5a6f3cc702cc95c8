"""Pins the CPU oracle (oracle/) against the reference's own known answers.

Every case in tests/golden/reference_kats.json names the reference test
(file:line) it was transcribed from.  If the oracle fails here it is not a
valid checker for the GPU path.
"""
import json
import os

import numpy as np
import pytest

from oracle import dccrg_oracle as O

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))


def leaves_with_refines(length, max_ref_lvl, refine):
    m = O.Mapping(length, max_ref_lvl)
    cells = set(range(1, int(np.prod(length)) + 1))
    for c in refine:
        cells.discard(c)
        cells |= set(m.get_all_children(c))
    return sorted(cells)


@pytest.mark.parametrize("case", GOLD["face_graph"], ids=lambda c: c["src"])
def test_face_graph_kat(case):
    g = O.Grid(case["length"], case["max_ref_lvl"], case["periodic"], 1,
               leaves_with_refines(case["length"], case["max_ref_lvl"], case["refine"]))
    for cell, ref in case["expect"].items():
        assert g.face_graph(int(cell)) == ref, (case["src"], cell)


@pytest.mark.parametrize("case", GOLD["face_neighbor_counts"], ids=lambda c: c["src"])
def test_face_neighbor_counts(case):
    g = O.Grid(case["length"], case["max_ref_lvl"], case["periodic"], 1,
               leaves_with_refines(case["length"], case["max_ref_lvl"], case["refine"]))
    for cell in g.cells():
        fn = g.face_neighbors_of(int(cell))
        assert len(fn) == case["count"], (case["src"], int(cell), fn)
        if "ids" in case:
            assert [i for i, _ in fn] == case["ids"][str(int(cell))]


def test_neighbor_list_length():
    c = GOLD["neighbor_list_length"]
    g = O.Grid(c["length"], 0, c["periodic"], c["hood_length"])
    for hood in c["hoods"]:
        items = g.hood_of if hood["items"] is None else np.array(hood["items"], dtype=np.int32)
        for cell in (1, 57, 1000):
            nof = g.find_neighbors_of(cell, items)
            nto = g.find_neighbors_to(cell, O.neighborhood_to(items))
            lof, lto = O.iteration_cache_lists(nof, nto)
            assert len(lof) == hood["nof"], hood["src"]
            assert len(lto) == hood["nto"], hood["src"]


def test_survey_facts():
    for f in GOLD["survey_facts"]:
        g = O.Grid(f["length"], f["max_ref_lvl"], f["periodic"], f["hood_length"],
                   leaves_with_refines(f["length"], f["max_ref_lvl"], f["refine"]))
        nof = g.find_neighbors_of(f["cell"])
        if "offsets" in f:
            got = [list(o) for i, o in nof if i == f["neighbor"]]
            assert got == f["offsets"], f["src"]
        if "neighbor_x_offsets_of_children_of_1" in f:
            kids = set(g.mapping.get_all_children(1))
            xs = sorted(set(o[0] for i, o in nof if i in kids))
            assert xs == f["neighbor_x_offsets_of_children_of_1"]
        if "offsets_all_equal" in f:
            got = [list(o) for i, o in nof if i == f["neighbor"]]
            assert len(got) >= f["min_repeats"]
            assert all(o == f["offsets_all_equal"] for o in got)
        if "axis_sequence" in f:
            got = [[i, o[0]] for i, o in nof if o[1] == 0 and o[2] == 0]
            assert got == f["axis_sequence"]


def _gol_run(case, steps):
    n = int(np.prod(case["length"]))
    alive = np.zeros(n, dtype=np.uint32)
    alive[np.array(case["initial_live"]) - 1] = 1
    return O.gol_reference_run(case["length"], case["periodic"], case["hood_length"], alive, steps)


def test_gol_kat_15x15():
    k = GOLD["gol_kat"]
    n = int(np.prod(k["length"]))
    alive = np.zeros(n, dtype=np.uint32)
    alive[np.array(k["initial_live"]) - 1] = 1
    lists = O.GolLists(k["length"], k["periodic"], k["hood_length"])
    count = np.zeros(n, dtype=np.uint32)
    for step in range(k["steps"]):
        # the test checks the state before the step is taken (game_of_life_test.cpp:371-381)
        live = set((np.nonzero(alive)[0] + 1).tolist())
        assert set(k["always_alive"]) <= live, step
        assert set(k["alive_even_steps" if step % 2 == 0 else "alive_odd_steps"]) <= live, step
        if str(step) in k["glider"]:
            assert set(k["glider"][str(step)]) <= live, step
        lists.step(alive, count)


def test_simple_gol_blinker():
    k = GOLD["simple_gol"]
    n = int(np.prod(k["length"]))
    alive = np.zeros(n, dtype=np.uint32)
    alive[np.array(k["initial_live"]) - 1] = 1
    lists = O.GolLists(k["length"], k["periodic"], k["hood_length"])
    count = np.zeros(n, dtype=np.uint32)
    for turn in range(k["turns"]):
        lists.step(alive, count)
        live = set((np.nonzero(alive)[0] + 1).tolist())
        assert set(k["always"]) <= live
        key = "even" if turn % 2 == 0 else "odd"
        assert set(k[f"after_{key}_turn_alive"]) <= live
        assert not (set(k[f"after_{key}_turn_dead"]) & live)


def test_line_kat_small():
    """The 1000x1000 line KAT's property, at a size the oracle runs in seconds."""
    k = GOLD["line_kat"]
    L = [64, 64, 1]
    y0 = 32
    n = L[0] * L[1]
    ids = np.arange(1, n + 1)
    alive = (((ids - 1) // L[0]) == y0).astype(np.uint32)
    steps = 16
    a, _ = O.gol_reference_run(L, k["periodic"], 1, alive, steps)
    rows = sorted(set(((np.nonzero(a)[0]) // L[0]).tolist()))
    assert rows == [y0 - steps, y0 + steps]
    assert int(a.sum()) == 2 * L[0]


def test_partition_block():
    # dccrg.hpp:8098-8145: 10 cells on 3 ranks -> 3,3,4 ... first ranks get fewer
    owners = [O.block_owner(10, 3, c) for c in range(1, 11)]
    assert owners == [0, 0, 0, 1, 1, 1, 2, 2, 2, 2]
    assert O.block_first_cell(10, 3, 2) == 7
    # fewer cells than processes: one cell each, trailing ranks empty
    assert [O.block_owner(2, 4, c) for c in (1, 2)] == [2, 3]


def test_mapping_hand_values():
    m = O.Mapping((10, 10, 1), 0)
    assert m.get_cell_from_indices((4, 5, 0), 0) == 55
    assert m.get_indices(55) == (4, 5, 0)
    m = O.Mapping((3, 3, 1), 1)
    # level-1 ids start at 10; cell 5's first child is at level-1 index (2,2,0)
    assert m.get_all_children(5) == [24, 25, 30, 31, 60, 61, 66, 67]
    assert m.get_refinement_level(9) == 0 and m.get_refinement_level(10) == 1
    assert m.get_refinement_level(82) == -1
    assert m.get_parent(67) == 5 and m.get_level_0_parent(67) == 5
    assert m.get_indices(0) == (O.ERROR_INDEX,) * 3
    assert m.get_cell_from_indices((6, 0, 0), 1) == O.ERROR_CELL
    # tests/geometry/README:4-24 runs this grid at max_ref_lvl 13, the largest possible
    assert O.max_possible_refinement_level((100, 200, 300)) == 13
