"""The incremental rebuild at the size the library picks it by itself (above
2^20 leaves): configs[2]'s adaptive advection loop on a 1000 x 1000 grid
(about 1.2 M leaves) stepped with the incremental neighbors_of, stencil rows
and neighbors_to, and again with every list rebuilt in full (test option
incremental = 0).  Leaf sets, densities and the neighbor lists of every leaf
must be identical after each step (the full rebuild is the path the oracle
parity tests pin at small sizes)."""
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
