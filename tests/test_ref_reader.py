"""The grid data file layout against the REFERENCE's own reader: files written
by the oracle restatement (oracle/dccrg_checkpoint.py; the device writes the
same bytes, tests/test_gpu_checkpoint.py) are parsed by tests/restart/
dc2vtk.cpp built where it lies -- its Mapping / Grid_Topology /
Cartesian_Geometry read() and the (id, offset) list and data that follow.
Header = u64 time step, cell data = u64 is_alive, as the restart test writes."""
import struct

import numpy as np
import pytest

import ref_reader as R
from oracle import dccrg_checkpoint as K
from oracle import dccrg_oracle as O

pytestmark = pytest.mark.skipif(not R.available(), reason="oracle/_ref/restart_dc2vtk is built where the reference is")


def refined_leaves(length, M, n, seed):
    rng = np.random.default_rng(seed)
    m = O.Mapping(length, M)
    n0 = int(np.prod(length))
    ref = set(int(v) for v in rng.choice(np.arange(1, n0 + 1), size=n, replace=False))
    leaves = []
    for c in range(1, n0 + 1):
        leaves += m.get_all_children(c) if c in ref else [c]
    return sorted(leaves)


@pytest.mark.parametrize("length,M,n_ref,P,start,l0", [
    ((6, 5, 4), 0, 0, 1, (0.0, 0.0, 0.0), (1.0, 1.0, 1.0)),
    ((6, 5, 4), 0, 0, 3, (-2.0, 0.5, 10.0), (0.25, 0.5, 2.0)),
    ((8, 8, 1), 2, 10, 2, (0.0, 0.0, 0.0), (0.125, 0.125, 0.125)),
    ((5, 3, 3), 1, 6, 4, (1.0, 2.0, 3.0), (0.5, 0.25, 1.0)),
])
def test_reference_reader_parses_oracle_files(tmp_path, length, M, n_ref, P, start, l0):
    cells = refined_leaves(length, M, n_ref, 3) if n_ref else list(range(1, int(np.prod(length)) + 1))
    n0 = int(np.prod(length))
    m = O.Mapping(length, M)
    alive = {c: int(O.splitmix64(np.array([c], dtype=np.uint64))[0] % 2) for c in cells}
    ranks = [[] for _ in range(P)]
    for c in cells:
        ranks[O.block_owner(n0, P, m.get_level_0_parent(c))].append((c, struct.pack("<Q", alive[c])))
    buf = K.write_grid_data(0, struct.pack("<Q", 42), length, M, 1, (True, False, True),
                            K.cartesian_geometry(start, l0), ranks)
    path = str(tmp_path / "grid.dc")
    open(path, "wb").write(buf)
    pts, got_alive = R.read_with_reference(path)
    order = [c for r in ranks for c, _ in r]
    assert got_alive.tolist() == [alive[c] for c in order]
    want = R.expected_corners(order, length, M, start, l0)
    np.testing.assert_allclose(pts, want, rtol=1e-5, atol=1e-9)  # dc2vtk prints 6 significant digits
