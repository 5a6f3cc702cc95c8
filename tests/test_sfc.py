"""Space-filling-curve placement of the level-0 cells (dccrg.hpp:8147-8220,
USE_SFC): the oracle's Hilbert restatement against the library's host keys,
and the curve's own properties.  sfc++ (the reference's curve) is not in the
reference tree, so the curve itself is parity-unpinned; the placement rule
(block counts along the curve, :8098-8114) is the reference's."""
import numpy as np
import pytest

import dccrg_amd as D
from dccrg_amd import _capi as X
from oracle import dccrg_oracle as O

BOXES = [(1, 1, 1), (2, 2, 2), (4, 4, 4), (5, 7, 3), (8, 8, 1), (33, 2, 17), (16, 16, 16), (100, 1, 1)]


@pytest.mark.parametrize("L", BOXES)
def test_library_keys_match_oracle(L):
    n = int(np.prod(L))
    out = np.zeros(n, dtype=np.uint64)
    ln = np.array(L, dtype=np.uint64)
    X.check(D.lib().dccrgx_hilbert_keys_host(ln.ctypes.data_as(X._u64p), out.ctypes.data_as(X._u64p)))
    key = O.hilbert_keys(L)
    assert np.array_equal(out, key)
    assert np.unique(key).size == n


@pytest.mark.parametrize("side", [2, 4, 8, 16])
def test_hilbert_curve_is_face_connected(side):
    L = (side, side, side)
    order = np.argsort(O.hilbert_keys(L))
    xyz = np.stack([order % side, (order // side) % side, order // (side * side)], 1)
    assert np.abs(np.diff(xyz, axis=0)).sum(1).max() == 1
    assert O.hilbert_keys(L).max() == side ** 3 - 1


@pytest.mark.parametrize("L,P", [((5, 7, 3), 4), ((10, 10, 10), 8), ((3, 1, 1), 5), ((9, 9, 9), 7)])
def test_owner_table_keeps_block_counts(L, P):
    n = int(np.prod(L))
    t = O.sfc_owner_table(L, P)
    counts = np.bincount(t, minlength=P)
    want = [sum(1 for c in range(1, n + 1) if O.block_owner(n, P, c) == r) for r in range(P)]
    assert counts.tolist() == want
    # each process holds one contiguous stretch of the curve
    key = O.hilbert_keys(L)
    for r in range(P):
        k = np.sort(key[t == r])
        if k.size:
            assert np.all(np.searchsorted(np.sort(key), k) == np.arange(k.size) + np.searchsorted(np.sort(key), k[0]))
