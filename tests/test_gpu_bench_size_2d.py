"""configs[1] checked at its full size with random state.

BASELINE configs[1] is the 2-D game of life on 16384 x 16384 x 1, hood 1,
periodic x and y (tests/game_of_life/scalability.cpp:85; z non-periodic so
the single layer is not its own neighbor), run by
dccrgx_gol_step through the vectorised row kernel k_gol26_rowv (1024-cell
x tiles per workgroup, row chunks along y).  The grid starts empty except for
random 24 x 24 patches where the indexing can go wrong -- the periodic x and y
wraps (corners and edges), the x tile seams and the y chunk seams -- and after
K steps every patch's window (padded by K + 1) is compared bit for bit with
the oracle's run (oracle/dccrg_oracle.c: the reference's neighbor lists and
B3/S23 rule) on a non-periodic box.  A device checksum of the whole grid must
equal the windows' sums: nothing outside them changed.  (The x-invariant line
KAT of scalability.cpp at this size is test_gpu_parity.py::test_line_kat_16384.)
"""
import numpy as np
import pytest

from oracle import dccrg_oracle as O

N = 16384
P = 24
K = 8
PAD = K + 1
M64 = (1 << 64) - 1

# lower corners (x, y); both axes wrap modulo N
PATCHES = [
    (16372, 16372),  # the corner: the window wraps in x and in y
    (0, 8000),       # low x edge, window wraps to x = N - 1
    (8188, 0),       # x tile seam 8192, low y edge wrapping to the last rows
    (1012, 5000),    # x tile seam 1024
    (3060, 16370),   # x seam 3072, high y edge wrapping to row 0
    (12276, 124),    # x seam 12288, y 128 (chunk seams are multiples of the chunk)
    (15350, 1020),   # x seam 15360, y 1024
    (6000, 4092),    # y 4096
    (9200, 12284),   # y 12288
    (16372, 2040),   # high x edge wrapping to x = 0, y 2048
]


def _window(p):
    """[lo, hi) per axis, unclipped (both axes wrap)."""
    return [(p[0] - PAD, p[0] + P + PAD), (p[1] - PAD, p[1] + P + PAD)]


def _disjoint(w1, w2):
    for ax in range(2):
        (a0, a1), (b0, b1) = w1[ax], w2[ax]
        if all(a1 <= b0 + s or b1 + s <= a0 for s in (-N, 0, N)):
            return True
    return False


def _ids(w):
    (x0, x1), (y0, y1) = w
    x = np.mod(np.arange(x0, x1, dtype=np.int64), N).astype(np.uint64)
    y = np.mod(np.arange(y0, y1, dtype=np.int64), N).astype(np.uint64)
    Y, X = np.meshgrid(y, x, indexing="ij")
    return (X + np.uint64(N) * Y + np.uint64(1)).ravel()


def test_windows_independent():
    ws = [_window(p) for p in PATCHES]
    for i in range(len(ws)):
        for j in range(i):
            assert _disjoint(ws[i], ws[j]), (PATCHES[i], PATCHES[j])


@pytest.mark.gpu
def test_gol_16384_squared_patches():
    import torch

    import dccrg_amd as D
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    ctx = D.Context(0, 0, 1)
    rng = np.random.default_rng(16384)
    g = (D.Dccrg().set_initial_length((N, N, 1)).set_neighborhood_length(1)
         .set_maximum_refinement_level(0).set_periodic(True, True, False).initialize(ctx))
    try:
        assert g.n_local == N * N
        for f in ("a", "b", "n"):
            g.add_field(f, np.uint32)
        expect = []
        for p in PATCHES:
            w = _window(p)
            dims = (w[0][1] - w[0][0], w[1][1] - w[1][0], 1)
            box = np.zeros((dims[1], dims[0]), dtype=np.uint32)  # [y, x]
            box[PAD:PAD + P, PAD:PAD + P] = rng.random((P, P)) < 0.25
            ids = _ids(w)
            sel = box.ravel() != 0
            g.write_cells("a", ids[sel], np.ones(int(sel.sum()), dtype=np.uint32))
            ra, rn = O.gol_reference_run(dims, (False, False, False), 1, box.ravel(), K)
            assert ra.sum() > 0
            expect.append((ids, ra, rn))
        cur, nxt = "a", "b"
        for _ in range(K):
            g.gol_step(cur, nxt, "n")
            cur, nxt = nxt, cur
        ctx.synchronize()
        sa = [0, 0]
        sn = [0, 0]
        for p, (ids, ra, rn) in zip(PATCHES, expect):
            got_a = np.concatenate(g.read_cells(cur, ids))
            got_n = np.concatenate(g.read_cells("n", ids))
            assert np.array_equal(got_a, ra), f"alive state differs in the window of patch {p}"
            assert np.array_equal(got_n, rn), f"neighbor counts differ in the window of patch {p}"
            mix = O.splitmix64(ids)
            with np.errstate(over="ignore"):
                sa[0] += int(ra.astype(np.uint64).sum())
                sa[1] = (sa[1] + int((ra.astype(np.uint64) * mix).sum(dtype=np.uint64))) & M64
                sn[0] += int(rn.astype(np.uint64).sum())
                sn[1] = (sn[1] + int((rn.astype(np.uint64) * mix).sum(dtype=np.uint64))) & M64
        assert g.checksum(cur) == tuple(sa)
        assert g.checksum("n") == tuple(sn)
    finally:
        g.close()
        ctx.close()
