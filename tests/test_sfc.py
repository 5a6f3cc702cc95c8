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


def _owners_from_library(L, P):
    n = int(np.prod(L))
    out = np.full(n, -7, dtype=np.int32)
    ln = np.array(L, dtype=np.uint64)
    X.check(D.lib().dccrgx_sfc_owners(None, ln.ctypes.data_as(X._u64p), P, out.ctypes.data_as(X._i32p)))
    return out


SFC_CASES = [((5, 7, 3), 4), ((64, 32, 16), 8), ((3, 1, 1), 5), ((100, 100, 1), 3), ((1, 1, 1), 1), ((1, 1, 1), 3),
             ((2, 2, 2), 8), ((2, 2, 2), 9), ((9, 9, 9), 7), ((33, 2, 17), 6), ((17, 1, 40), 12), ((31, 29, 23), 16),
             ((128, 1, 1), 128), ((7, 7, 7), 343), ((1, 50, 3), 2), ((40, 40, 40), 64)]


@pytest.mark.parametrize("L,P", SFC_CASES)
def test_cut_keys_give_the_oracle_owner_table(L, P):
    """The placement kept as P - 1 cut keys (sfc.hip: counted over the Hilbert
    octree, no per-cell table) gives every level-0 cell the owner of the
    oracle's sort-based table (dccrg.hpp:8147-8220 with :8098-8114's counts)."""
    assert np.array_equal(_owners_from_library(L, P), O.sfc_owner_table(L, P))


@pytest.mark.parametrize("L,P", SFC_CASES)
def test_cut_keys_are_the_first_keys_of_each_process(L, P):
    n = int(np.prod(L))
    cuts = np.zeros(max(P - 1, 1), dtype=np.uint64)
    ln = np.array(L, dtype=np.uint64)
    X.check(D.lib().dccrgx_sfc_cuts(ln.ctypes.data_as(X._u64p), P, cuts.ctypes.data_as(X._u64p)))
    skey = np.sort(O.hilbert_keys(L))
    for r in range(1, P):
        first = [c for c in range(1, n + 1) if O.block_owner(n, P, c) == r]
        want = skey[first[0] - 1] if first else np.uint64(2 ** 64 - 1)
        # a process with no cells repeats the next one's cut (the owner count skips it)
        if not first:
            later = [c for c in range(1, n + 1) if O.block_owner(n, P, c) > r]
            want = skey[later[0] - 1] if later else np.uint64(2 ** 64 - 1)
        assert cuts[r - 1] == want, (r, cuts[r - 1], want)


def test_cut_keys_of_a_large_grid_need_no_cell_walk():
    """2^30 level-0 cells (past what an owner table would hold cheaply): the
    cuts come from the octree count alone; each cut key's cell has exactly the
    block partition's number of cells before it on the curve (checked by the
    oracle-independent count over sub-cubes of a coarser curve)."""
    L, P = (1024, 1024, 1024), 8
    cuts = np.zeros(P - 1, dtype=np.uint64)
    ln = np.array(L, dtype=np.uint64)
    X.check(D.lib().dccrgx_sfc_cuts(ln.ctypes.data_as(X._u64p), P, cuts.ctypes.data_as(X._u64p)))
    # a power-of-two cube: every key is a cell, so process r starts at key r * n / P
    n = 1024 ** 3
    assert cuts.tolist() == [r * n // P for r in range(1, P)]
