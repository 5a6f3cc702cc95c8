"""The bench's synthetic grids are the ones the tests check: bench.py builds
them without the oracle (the product path never imports it), so their
construction is checked here against the oracle's."""
import numpy as np

import bench
from oracle import dccrg_oracle as O
from test_oracle_poisson import poisson3d_leaves


def test_bench_poisson_grid_is_poisson3d():
    m, leaves = poisson3d_leaves()
    ids, idx, lvl = bench.poisson3d_leaves()
    assert ids.tolist() == leaves
    oi, ol = m.ids_to_indices(ids)
    assert np.array_equal(oi.astype(np.float64), idx) and np.array_equal(ol, lvl)


def test_bench_advection_grid_is_balanced():
    """Small version of the advection snapshot: every leaf's face neighbors
    are within one level, and the leaves tile the domain."""
    n = 24
    leaves = bench.advection_leaves(n=n, r1=0.3, r2=0.15)
    m = O.Mapping((n, n, 1), 2)
    lvl = np.array([m.get_refinement_level(int(c)) for c in leaves])
    assert np.isclose(np.sum(8.0 ** -lvl), n * n)  # volume
    assert set(np.unique(lvl)) == {0, 1, 2}
    g = O.Grid((n, n, 1), 2, (True, True, False), 0, leaves.tolist())
    for c in leaves[:: max(1, len(leaves) // 400)]:
        for nb, _ in g.find_neighbors_of(int(c)):
            assert abs(m.get_refinement_level(nb) - m.get_refinement_level(int(c))) <= 1
            assert g.exists(nb)
