"""The incremental rebuild at the size the library picks it by itself (above
2^20 leaves): configs[2]'s adaptive advection loop on a 1000 x 1000 grid
(about 1.2 M leaves) stepped with the incremental neighbors_of, stencil rows
and neighbors_to, and again with every list rebuilt in full (test option
incremental = 0).  Leaf sets, densities and the neighbor lists of every leaf
must be identical after each step (the full rebuild is the path the oracle
parity tests pin at small sizes)."""
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from dccrg_amd import advection as A  # noqa: E402
from dccrg_amd.grid import set_test_option  # noqa: E402

NX, M, STEPS = 1000, 2, 3
REL, THR, SENS, CFL = 0.006, 0.25, 0.5, 0.5


def run(incremental):
    set_test_option("incremental", incremental)
    try:
        ctx = D.Context(0, 0, 1)
        g = (D.Dccrg().set_initial_length((NX, NX, 1)).set_maximum_refinement_level(M)
             .set_periodic(True, True, False).set_neighborhood_length(0).initialize(ctx))
        g.add_advection_fields()
        geom = A.geometry_2d(g)
        A.initialize(g, geom)
        for _ in range(M):
            A.adapt_grid(g, geom, *A.check_for_adaptation(g, REL / M, THR, SENS))
            A.initialize(g, geom)
        dt = g.max_time_step()
        g.update_copies_of_remote_neighbors(fields=list(A.ALL))
        states = []
        for _ in range(STEPS):
            g.update_copies_of_remote_neighbors(fields=["density"])
            sets = A.check_for_adaptation(g, REL / M, THR, SENS)
            g.advect_step(CFL * dt)
            A.adapt_grid(g, geom, *sets)
            dt = g.max_time_step()
            cells = g.local_cells()
            row, ids, off = g.neighbors_of(cells)
            trow, tids = g.neighbors_to(cells)
            states.append((cells.copy(), g.read_local("density").copy(), row.copy(), ids.copy(), off.copy(),
                           trow.copy(), tids.copy()))
        g.close()
        ctx.close()
        return states
    finally:
        set_test_option("incremental", None)


def test_incremental_rebuild_equals_full_rebuild_at_scale():
    inc = run(1)
    full = run(0)
    assert inc[0][0].size > (1 << 20), "the grid must exceed the incremental threshold"
    names = ("leaves", "density", "neighbors_of rows", "neighbors_of ids", "neighbors_of offsets",
             "neighbors_to rows", "neighbors_to ids")
    for step, (a, b) in enumerate(zip(inc, full)):
        for name, x, y in zip(names, a, b):
            assert x.shape == y.shape and np.array_equal(x, y), (step, name)


def _refine_one(length, idx0):
    """A uniform grid (hood length 1, one level) with the level-0 cell at
    idx0 refined: the grid, its field "a" (low id bits, written before)."""
    ctx = D.Context(0, 0, 1)
    g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(1)
         .set_periodic(False, False, False).set_neighborhood_length(1).initialize(ctx))
    g._keep = ctx
    g.add_field("a", np.uint32)
    g.write_local("a", (g.local_cells() & 0xFFFFFFFF).astype(np.uint32))
    assert g.info.uniform == 1
    c = g.mapping.get_cell_from_indices(tuple(2 * v for v in idx0), 0)  # indices in level-1 units
    assert g.refine_completely(c) == 1
    t0 = time.perf_counter()
    new = g.stop_refining()
    dt = time.perf_counter() - t0
    assert g.info.uniform == 0
    return g, c, new, dt


def test_refine_one_cell_of_a_large_uniform_grid():
    """The uniform -> explicit switch at 2^24 level-0 cells (one rank: the
    leaf list and the move plan are generated on the device, amr.hip
    ensure_explicit).  Every unchanged cell keeps its data; around the
    refined cell the neighbor lists equal those of a 5^3 grid refined at its
    centre, translated (hood length 1 reaches one level-0 cell, so the patch
    sees no boundary in either grid)."""
    L, at = 256, (100, 37, 200)
    big, cb, new_b, dt = _refine_one((L, L, L), at)
    small, cs, new_s, _ = _refine_one((5, 5, 5), (2, 2, 2))
    print(f"refine of one cell of a {L}^3 uniform grid: {dt * 1e3:.1f} ms")
    N = L ** 3
    loc = big.local_cells()
    assert loc.size == N - 1 + 8 and new_b.size == 8
    vals = big.read_local("a")
    keep = ~np.isin(loc, new_b)
    assert np.array_equal(vals[keep], (loc[keep] & 0xFFFFFFFF).astype(np.uint32))
    assert np.all(vals[~keep] == 0)
    # the patch: the refined cell's children and its 26 level-0 neighbors
    sl = small.local_cells()
    idx, lvl = small.mapping.levels_and_indices(sl)
    span = 2  # a level-0 cell in max-level (level-1) index units
    inner = np.all((idx >= 1 * span) & (idx < 4 * span), axis=1)
    patch = sl[inner]
    assert patch.size == 26 + 8
    shift = np.array([(a - 2) * span for a in at], dtype=np.uint64)

    def tr(ids):
        i, l = small.mapping.levels_and_indices(ids)
        return np.array([big.mapping.get_cell_from_indices(tuple(v + shift), int(k)) for v, k in zip(i, l)],
                        dtype=np.uint64)

    assert np.array_equal(np.sort(tr(new_s)), np.sort(new_b))
    rs, ids_s, off_s = small.neighbors_of(patch)
    rb, ids_b, off_b = big.neighbors_of(tr(patch))
    assert np.array_equal(rs, rb) and np.array_equal(off_s, off_b)
    assert np.array_equal(tr(ids_s), ids_b.astype(np.uint64))
    trs, tids_s = small.neighbors_to(patch)
    trb, tids_b = big.neighbors_to(tr(patch))
    assert np.array_equal(trs, trb)
    assert np.array_equal(tr(tids_s), tids_b.astype(np.uint64))
    for g in (big, small):
        g.close()
