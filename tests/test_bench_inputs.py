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
