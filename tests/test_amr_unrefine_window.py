"""CPU: override_unrefines' face-graph walk (dccrg.hpp:9935-10124, restated
literally in oracle/dccrg_amr.py _override_unrefines) equals the window test
the device runs by default (amr_dev.hip k_ou_check): an unrefine survives iff
every sibling is a leaf outside cells_to_refine / cells_not_to_unrefine and no
leaf overlapping the parent's neighborhood windows is finer than the unrefined
cell, or of its level and to be refined.  Checked for every pending unrefine
of random request sequences, hood lengths 0-2, periodic and not, up to three
levels; in the hood 0 and 1 cases some unrefines are overridden (a refine
two or three steps from the group, or one it induces, lands in the parent's
windows).  The GPU suite checks the device decisions against the oracle too."""
import numpy as np
import pytest

from oracle.dccrg_amr import ERROR_CELL, AmrOracle


def _walk(o, unrefined, R, nnu):
    parent = o.mapping.get_parent(unrefined)
    if any(s != ERROR_CELL and (s in R or s in nnu) for s in o.mapping.get_all_children(parent)):
        return False
    ul = o.level(unrefined)
    processed, process = set(), set(o.face(unrefined))
    process.discard(ERROR_CELL)
    while process:
        nxt = min(process)
        processed.add(nxt)
        process.discard(nxt)
        for n in o.face(nxt):
            if n == ERROR_CELL or n in processed:
                continue
            if o.is_neighbor(parent, n):
                process.add(n)
            else:
                processed.add(n)
        rl = o.level(nxt)
        if rl > ul or (rl == ul and nxt in R):
            return False
    return True


def _window(o, unrefined, R, nnu):
    parent = o.mapping.get_parent(unrefined)
    ul = o.level(unrefined)
    for s in o.mapping.get_all_children(parent):
        if s not in o.leaves or s in R or s in nnu:
            return False
    for n in o.parent_window_leaves(parent):
        nl = o.level(n)
        if nl > ul or (nl == ul and n in R):
            return False
    return True


CASES = [((4, 4, 3), 2, (False, False, False), 1, 0), ((4, 3, 3), 2, (True, True, True), 1, 1),
         ((5, 4, 2), 2, (True, False, False), 0, 2), ((3, 3, 3), 2, (False, True, True), 2, 3),
         ((3, 2, 2), 3, (True, True, False), 1, 4), ((6, 1, 1), 3, (False, False, False), 1, 5),
         ((2, 2, 2), 2, (True, True, True), 2, 6)]


@pytest.mark.parametrize("length,M,per,hood,seed", CASES)
def test_walk_equals_window_test(length, M, per, hood, seed):
    checked = survived = 0
    for rnd in range(21):
        if rnd % 7 == 0:  # three request sequences from a uniform grid
            rng = np.random.default_rng(10 * seed + rnd // 7)
            o = AmrOracle(length, M, per, hood, 1)
        # unrefines first, then refines: a refine reaching a parent's windows
        # but not the group (or induced by one) overrides an unrefine
        fine = [c for c in o.cells() if o.level(c) > 0]
        for c in rng.permutation(fine)[: max(1, len(fine) // 2)]:
            o.unrefine_completely(0, int(c))
        cells = o.cells()
        for c in rng.choice(cells, min(len(cells), 4), replace=False):
            o.refine_completely(0, int(c))
        pend = sorted(o.to_unrefine[0])
        for u in (rng.choice(pend, min(len(pend), 6), replace=False) if pend else []):
            # a leaf a few steps away: its refine (or one it induces) may land
            # in the parent's windows without touching the group
            x = int(u)
            for _ in range(int(rng.integers(2, 4))):
                nb = o.nof(x)
                x = int(nb[rng.integers(len(nb))]) if nb else x
            o.refine_completely(0, x)
        for c in rng.choice(o.cells(), 2, replace=False):
            if rng.integers(3) == 0:
                o.dont_unrefine(0, int(c))
        o._override_refines()
        o._induce_refines()
        R, nnu = set(o.to_refine[0]), set(o.not_to_unrefine[0])
        for u in sorted(o.to_unrefine[0]):
            w = _walk(o, u, R, nnu)
            assert w == _window(o, u, R, nnu), (rnd, u)
            checked += 1
            survived += w
        o._override_unrefines()
        o._execute_refines()
    assert checked > 0 and (survived < checked or hood != 1), (checked, survived)
