"""The AMR restatement (oracle/dccrg_amr.py) against the reference's own
refinement tests (tests/refine/*.cpp), which state their expected outcomes in
code, and against the 2:1 balance invariant those tests check."""
import numpy as np
import pytest

from oracle.dccrg_amr import AmrOracle


def corner_leaf(o: AmrOracle) -> int:
    """refine_completely_at / unrefine_completely_at of a coordinate just
    inside the grid's starting corner: the smallest existing cell at indices
    (0, 0, 0) (dccrg.hpp:3401-3460 with the corner of
    tests/refine/refine_simple.cpp:97-101)."""
    for lvl in range(o.M, -1, -1):
        c = o.mapping.get_cell_from_indices((0, 0, 0), lvl)
        if c in o.leaves:
            return c
    raise AssertionError


@pytest.mark.parametrize("P", [1, 2, 3])
def test_dont_refine_cases(P):
    """tests/refine/dont_refine.cpp: cell 1's first child (id 4) never
    appears, whether the refine is direct, from a face neighbor, from a
    further neighbor or from the furthest one."""
    o = AmrOracle((3, 1, 1), -1, hood_length=1, comm_size=P)
    r1 = o.owner(1)
    o.dont_refine(r1, 1)
    o.refine_completely(r1, 1)
    o.stop_refining()
    assert 4 not in o.leaves

    o = AmrOracle((3, 1, 1), -1, hood_length=1, comm_size=P)
    o.refine_completely(o.owner(2), 2)
    o.stop_refining()
    o.dont_refine(o.owner(1), 1)
    o.refine_completely(o.owner(6), 6)
    o.stop_refining()
    assert 4 not in o.leaves and 6 in o.leaves
    o.dont_refine(o.owner(1), 1)
    o.refine_completely(o.owner(7), 7)
    o.stop_refining()
    # 7 lies in cell 1's neighborhood (hood length 1 reaches all of cell 2),
    # so the persisting dont_refine spread (dccrg.hpp:10176) blocks it too
    assert 4 not in o.leaves and 7 in o.leaves
    assert o.max_level_difference() <= 1

    o = AmrOracle((3, 1, 1), -1, hood_length=1, comm_size=P)
    o.refine_completely(o.owner(3), 3)
    o.stop_refining()
    o.dont_refine(o.owner(1), 1)
    o.refine_completely(o.owner(8), 8)
    o.stop_refining()
    assert 2 not in o.leaves  # induced by the refined neighbor 8
    o.refine_completely(o.owner(37), 37)
    o.stop_refining()
    assert 4 not in o.leaves and 1 in o.leaves
    assert o.max_level_difference() <= 1


@pytest.mark.parametrize("P", [1, 2])
def test_refine_simple_balance(P):
    """tests/refine/refine_simple.cpp:91-121: refining the corner cell three
    times keeps every neighbor within one refinement level."""
    o = AmrOracle((2, 1, 1), -1, hood_length=1, comm_size=P)
    for step in range(3):
        c = corner_leaf(o)
        assert o.refine_completely(o.owner(c), c)
        new = o.stop_refining()
        assert sum(len(x) for x in new) >= 8
        assert o.max_level_difference() <= 1
        assert corner_leaf(o) == o.mapping.get_all_children(c)[0]
    assert o.level(corner_leaf(o)) == 3


def test_unrefine_simple_sequence():
    """tests/refine/unrefine_simple.cpp: four corner refines then four corner
    unrefines (max_ref_lvl 5).  The reference test only requires the run to
    complete; the corner level trajectory below is the restatement's (the
    induced refines around the corner keep the level-2 corner's siblings
    refined, so its unrefine is refused by :2621-2624)."""
    o = AmrOracle((2, 1, 1), 5, hood_length=1)
    levels = []
    for step in range(8):
        c = corner_leaf(o)
        if step < 4:
            assert o.refine_completely(0, c)
        else:
            o.unrefine_completely(0, c)
        o.stop_refining()
        assert o.max_level_difference() <= 1
        levels.append(o.level(corner_leaf(o)))
    assert levels == [1, 2, 3, 4, 3, 2, 2, 2]


def test_unrefine_blocked_by_refine_and_dont_unrefine():
    """unrefine_completely: no effect when a sibling is to be refined
    (dccrg.hpp:2621-2629) or marked by dont_unrefine (:2701-2760), and the
    removed cells are reported with their parent re-created (:10437-10520)."""
    o = AmrOracle((4, 4, 1), 2, periodic=(True, True, False), hood_length=1)
    o.refine_completely(0, 6)
    o.stop_refining()
    kids = o.mapping.get_all_children(6)
    o.refine_completely(0, kids[0])
    o.unrefine_completely(0, kids[1])
    o.stop_refining()
    assert kids[1] in o.leaves and kids[0] not in o.leaves
    o = AmrOracle((4, 4, 1), 2, hood_length=1)
    o.refine_completely(0, 6)
    o.stop_refining()
    kids = o.mapping.get_all_children(6)
    o.dont_unrefine(0, kids[3])
    o.unrefine_completely(0, kids[0])
    o.stop_refining()
    assert kids[0] in o.leaves
    o.unrefine_completely(0, kids[0])
    o.stop_refining()
    assert 6 in o.leaves and o.get_removed_cells(0) == sorted(kids)


def test_random_sequences_stay_balanced():
    rng = np.random.default_rng(3)
    o = AmrOracle((5, 4, 3), 2, periodic=(True, False, True), hood_length=1, comm_size=2)
    for _ in range(4):
        cells = o.cells()
        for c in rng.choice(cells, 6, replace=False):
            c = int(c)
            r = o.owner(c)
            k = rng.integers(3)
            if k == 0:
                o.refine_completely(r, c)
            elif k == 1:
                o.unrefine_completely(r, c)
            else:
                o.dont_unrefine(r, c)
        o.stop_refining()
        assert o.max_level_difference() <= 1
