"""GPU: refinement inside a uniform grid (dccrg_amd/csrc/hybrid.hip, the first
slice of the hybrid layout).  A one-process uniform grid whose explicit form
would not fit the device refines in place: level-0 cells keep the implicit
slab layout and closed-form rows, the refined cells' children get slots after
it, and the leaves whose rows involve a refined cell keep rows built by the
explicit machinery over a box around them.

Checks: (1) with the test option "hybrid" forcing the path on small grids,
the hybrid grid equals the same grid refined through the explicit layout
(itself oracle-checked in test_gpu_amr.py) -- leaves, new and removed cells,
request results, every leaf's neighbors_of / neighbors_to and several
game-of-life steps -- over two rounds of refines, then two rounds of
unrefines back to level 0 (one group kept by dont_unrefine, a new refine
beside them), periodic and not, hood lengths 0, 1, 2; (2) a 1024^3 grid (1.07e9
cells, over the explicit layout's ~2.4e8-cell limit) refines one cell: the
lists and the game of life around it equal a small grid refined the same way,
a patch far from it equals a small uniform grid, and a whole-grid checksum
equals the windows' sums (no other cell written)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from dccrg_amd.grid import set_test_option  # noqa: E402


def _grid(length, per, hood, M=1):
    ctx = D.Context(0, 0, 1)
    g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
         .set_neighborhood_length(hood).initialize(ctx))
    g._keep = ctx
    for f in ("a", "b", "n"):
        g.add_field(f, np.uint32)
    return g


def _gol(g, steps):
    cur, nxt = "a", "b"
    for _ in range(steps):
        g.gol_step(cur, nxt, "n")
        cur, nxt = nxt, cur
    return cur


CASES = [((12, 10, 8), (False, False, False), 1), ((12, 10, 8), (True, True, True), 1),
         ((9, 9, 9), (True, False, True), 0), ((14, 12, 10), (False, True, False), 2),
         ((6, 5, 7), (True, True, True), 1)]


@pytest.mark.parametrize("length,per,hood", CASES)
def test_hybrid_equals_explicit_refinement(length, per, hood):
    rng = np.random.default_rng(sum(length) + hood)
    n0 = int(np.prod(length))
    alive = (rng.random(n0) < 0.35).astype(np.uint32)
    grids = []
    try:
        for hybrid in (True, False):
            set_test_option("hybrid", 1 if hybrid else None)
            g = _grid(length, per, hood)
            g.write_local("a", alive)
            grids.append(g)
        hy, ex = grids
        picks = rng.choice(np.arange(1, n0 + 1), size=(3, 4), replace=False)
        refined = []
        for rnd in range(4):
            if rnd < 2:
                cells = [int(c) for c in picks[rnd]]
                if rnd == 1:  # a neighbor of an earlier refined cell too (adjacent refined blocks)
                    cells.append(int(picks[0][0]) + 1 if (int(picks[0][0]) % length[0]) else int(picks[0][0]) - 1)
                for g in grids:
                    for c in cells:
                        assert g.refine_completely(c)
                refined += cells
            else:
                # unrefines: one child of a group, every child of another, a
                # group kept by dont_unrefine, and (round 2) a new refine
                # beside them; round 3 unrefines what is left
                groups = sorted(set(refined))
                if rnd == 2:
                    un, keep = groups[:3], groups[3]
                else:
                    un, keep = groups, None
                for g in grids:
                    res = []
                    for k, p in enumerate(un):
                        kids = [int(x) for x in g.mapping.get_all_children(p)]
                        for c in (kids if k == 1 else kids[k % 8:k % 8 + 1]):
                            res.append(g.unrefine_completely(c))
                    if keep is not None:
                        kids = [int(x) for x in g.mapping.get_all_children(keep)]
                        res.append(g.unrefine_completely(kids[2]))
                        res.append(g.dont_unrefine(kids[5]))
                    if rnd == 2:
                        res.append(g.refine_completely(int(picks[2][0])))
                    g._res = res
                assert hy._res == ex._res
                refined = [c for c in groups if c not in un]
                if rnd == 2:
                    refined.append(int(picks[2][0]))
            set_test_option("hybrid", 1)
            new_h = hy.stop_refining()
            set_test_option("hybrid", None)
            new_e = ex.stop_refining()
            assert hy.info.uniform == 2 and ex.info.uniform == 0
            assert np.array_equal(np.sort(new_h), np.sort(new_e))
            assert np.array_equal(np.sort(hy.get_removed_cells()), np.sort(ex.get_removed_cells()))
            if rnd >= 2:
                assert len(ex.get_removed_cells()) > 0
            leaves = ex.local_cells()
            assert np.array_equal(hy.local_cells(), leaves)
            assert hy.info.n_local == leaves.size
            rh, ih, oh = hy.neighbors_of(leaves)
            re_, ie, oe = ex.neighbors_of(leaves)
            assert np.array_equal(rh, re_) and np.array_equal(ih, ie) and np.array_equal(oh, oe)
            th, tih = hy.neighbors_to(leaves)
            te, tie = ex.neighbors_to(leaves)
            assert np.array_equal(th, te) and np.array_equal(tih, tie)
            # the same data in both (children start at 0 in both), then the game of life
            vals = ex.read_local("a")
            assert np.array_equal(hy.read_local("a"), vals)
            for g in grids:
                cur = _gol(g, 3)
                if cur != "a":
                    g.write_local("a", g.read_local(cur))
            assert np.array_equal(hy.read_local("a"), ex.read_local("a"))
            assert np.array_equal(hy.read_local("n"), ex.read_local("n"))
            assert hy.checksum("a") == ex.checksum("a")
    finally:
        set_test_option("hybrid", None)
        for g in grids:
            g.close()


def test_unsupported_calls_refuse_on_hybrid_grids():
    set_test_option("hybrid", 1)
    g = _grid((6, 6, 6), (False, False, False), 1)
    try:
        g.refine_completely(50)
        g.stop_refining()
        assert g.info.uniform == 2
        child = int(g.get_new_cells()[0])
        from dccrg_amd import _capi as X
        with pytest.raises(D.DccrgxError) as e:  # a level-1 refine: not in this slice
            g.refine_completely(child)
        assert e.value.code == X.DCCRGX_ESTATE
        with pytest.raises(D.DccrgxError) as e:
            g.add_neighborhood(5, [[1, 0, 0], [-1, 0, 0]])
        assert e.value.code == X.DCCRGX_ESTATE
    finally:
        set_test_option("hybrid", None)
        g.close()


def test_refine_one_cell_of_a_grid_beyond_the_explicit_layout():
    """1024^3 = 1.07e9 level-0 cells, hood 1, one level: the explicit layout
    would need ~1.3 TB; the grid refines in place.  Patches: around the
    refined cell (against a 16^3 grid refined at the same relative place) and
    far from it (against a 16^3 uniform grid), K steps of the game of life."""
    L, at, far, P, K = 1024, (517, 300, 811), (100, 900, 40), 16, 3
    rng = np.random.default_rng(7)
    big = _grid((L, L, L), (False, False, False), 1)
    small_r = _grid((P, P, P), (False, False, False), 1)
    small_u = _grid((P, P, P), (False, False, False), 1)
    try:
        mb, ms = big.mapping, small_r.mapping
        c = P // 2

        def ids_of(origin, m, lo, hi):
            z, y, x = np.meshgrid(np.arange(lo, hi), np.arange(lo, hi), np.arange(lo, hi), indexing="ij")
            idx = np.stack([x.ravel() + origin[0], y.ravel() + origin[1], z.ravel() + origin[2]], 1)
            return np.array([m.get_cell_from_indices(tuple(int(v) * 2 for v in r), 0) for r in idx], dtype=np.uint64)

        # live cells in a 6^3 block around each patch centre (K steps spread
        # them at most K cells: the 16^3 small grids hold everything)
        blk_small = ids_of((0, 0, 0), ms, c - 3, c + 3)
        vals = (rng.random(blk_small.size) < 0.4).astype(np.uint32)
        o_at = tuple(a - c for a in at)
        o_far = tuple(a - c for a in far)
        big.write_cells("a", ids_of(o_at, mb, c - 3, c + 3), vals)
        big.write_cells("a", ids_of(o_far, mb, c - 3, c + 3), vals)
        for g in (small_r, small_u):
            g.write_cells("a", blk_small, vals)
        rc_big = mb.get_cell_from_indices(tuple(2 * v for v in at), 0)
        rc_small = ms.get_cell_from_indices((2 * c, 2 * c, 2 * c), 0)
        assert big.refine_completely(rc_big) and small_r.refine_completely(rc_small)
        new_b = big.stop_refining()
        small_r.stop_refining()
        assert big.info.uniform == 2 and new_b.size == 8
        assert big.info.n_local == L ** 3 - 1 + 8

        def tr(ids, origin):  # small-grid ids -> big-grid ids
            i, lv = ms.levels_and_indices(ids)
            sh = np.array([2 * o for o in origin], dtype=np.int64)
            return np.array([mb.get_cell_from_indices(tuple(int(a) for a in (v + sh)), int(k)) for v, k in zip(i, lv)],
                            dtype=np.uint64)

        # neighbor lists of the patch around the refined cell
        sl = small_r.local_cells()
        si, slv = ms.levels_and_indices(sl)
        near = sl[np.all((si >= 2 * (c - 2)) & (si < 2 * (c + 3)), axis=1)]
        rs, ids_s, off_s = small_r.neighbors_of(near)
        rb, ids_b, off_b = big.neighbors_of(tr(near, o_at))
        assert np.array_equal(rs, rb) and np.array_equal(off_s, off_b)
        assert np.array_equal(tr(ids_s, o_at), ids_b)
        # K steps everywhere
        cb, cr, cu = _gol(big, K), _gol(small_r, K), _gol(small_u, K)
        inner_r = small_r.local_cells()
        inner_u = small_u.local_cells()
        for name_b, name_s, g, inner, origin in ((cb, cr, small_r, inner_r, o_at), (cb, cu, small_u, inner_u, o_far)):
            want = np.concatenate(g.read_cells(name_s, inner))
            got = np.concatenate(big.read_cells(name_b, tr(inner, origin)))
            assert np.array_equal(got, want), origin
            want_n = np.concatenate(g.read_cells("n", inner))
            got_n = np.concatenate(big.read_cells("n", tr(inner, origin)))
            assert np.array_equal(got_n, want_n), origin
        # nothing else alive: the whole grid's sums are the two windows' sums
        sb = big.checksum(cb)
        s_r, s_u = small_r.checksum(cr), small_u.checksum(cu)
        assert sb[0] == s_r[0] + s_u[0]
        # unrefine back to level 0 (one child's request takes the group): the
        # children go, the parent comes back value-initialised, and a step of
        # the game of life around it equals the small grid's
        kb = [int(x) for x in mb.get_all_children(rc_big)]
        ks = [int(x) for x in ms.get_all_children(rc_small)]
        assert big.unrefine_completely(kb[3]) and small_r.unrefine_completely(ks[3])
        assert big.stop_refining().size == 0
        small_r.stop_refining()
        assert np.array_equal(np.sort(big.get_removed_cells()), np.sort(np.array(kb, dtype=np.uint64)))
        assert big.info.n_local == L ** 3
        assert int(np.concatenate(big.read_cells(cb, np.array([rc_big], dtype=np.uint64)))[0]) == 0
        nxt = "a" if cb == "b" else "b"
        big.gol_step(cb, nxt, "n")
        small_r.gol_step(cr, nxt, "n")
        inner_r = small_r.local_cells()
        assert inner_r.size == P ** 3
        for name in (nxt, "n"):
            want = np.concatenate(small_r.read_cells(name, inner_r))
            got = np.concatenate(big.read_cells(name, tr(inner_r, o_at)))
            assert np.array_equal(got, want), name
    finally:
        for g in (big, small_r, small_u):
            g.close()
