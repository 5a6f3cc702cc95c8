"""The headline kernel checked at the size the bench quotes it on.

bench.py times the 3-D game of life on 2048 x 2048 x 2048 (8.59e9 cells, more
than 2^32), hood 1, periodic z, through dccrgx_gol_step (halo start, inner,
wait, outer: tests/game_of_life/scalability3d.cpp:122-166).  A full-grid CPU
comparison is out of reach, so the grid starts empty except for random 24^3
patches at the places where the kernel's indexing can go wrong:
- the A/B tile seams of the stencil (256-cell A tiles, 32-row B tiles) and the
  C chunk seams (128 slices per workgroup at this size),
- the non-periodic x/y edges and the first/last planes with the periodic z
  wrap between them,
- planes whose linear cell index exceeds 2^32, and the plane where it crosses.
Live cells spread by at most one cell per step, so after K steps a patch's
state lies within K cells of it; every patch is compared, bit for bit, with
the oracle's run (oracle/dccrg_oracle.c, the reference's neighbor lists and
B3/S23 rule) on the patch's window padded by K + 1 cells (a non-periodic box:
cells beyond are dead in both).  A device checksum of the whole grid (sum and
id-weighted sum over all 8.59e9 cells) must equal the windows' sums, so no
cell outside the windows was written either.
"""
import numpy as np
import pytest

from oracle import dccrg_oracle as O

N = 2048       # cells per axis (bench.py default, BASELINE configs[3] per GPU)
P = 24         # patch edge
K = 8          # steps
PAD = K + 1
M64 = (1 << 64) - 1

# lower corners (x, y, z); z wraps modulo N
PATCHES = [
    (0, 0, 2036),        # x/y low edges; last plane -> first plane through the periodic z wrap
    (2024, 2024, 1500),  # x/y high edges, linear index > 2^32
    (244, 1012, 1140),   # A seam 256, B seam 1024, C chunk seam 1152, > 2^32
    (1780, 52, 1012),    # A seam 1792, B seam 64, crosses plane 1024 (linear index 2^32)
    (0, 0, 1012),        # holds linear index 2^32 itself (x = y = 0, z = 1024)
    (2024, 2024, 1012),  # holds 2^32 - 1 (x = y = 2047, z = 1023), its +z neighbors beyond 2^32
    (500, 2024, 628),    # B high edge, C chunk seam 640
    (1012, 500, 116),    # C chunk seam 128
    (1516, 1300, 1780),  # A seam 1536, B seam 1312, > 2^32
    (244, 2024, 1780),   # A seam 256 at the B high edge, > 2^32
]


def _window(p):
    """[lo, hi) per axis: x, y clipped to the non-periodic grid; z unclipped (wraps)."""
    x0, y0, z0 = p
    return [(max(0, x0 - PAD), min(N, x0 + P + PAD)), (max(0, y0 - PAD), min(N, y0 + P + PAD)),
            (z0 - PAD, z0 + P + PAD)]


def _disjoint(w1, w2):
    for ax in range(3):
        (a0, a1), (b0, b1) = w1[ax], w2[ax]
        if ax < 2:
            if a1 <= b0 or b1 <= a0:
                return True
        else:  # periodic: disjoint unless some shift by N overlaps
            if all(a1 <= b0 + s or b1 + s <= a0 for s in (-N, 0, N)):
                return True
    return False


def _ids(w):
    """grid ids of a window, ordered like the oracle box (x fastest)."""
    (x0, x1), (y0, y1), (z0, z1) = w
    x = np.arange(x0, x1, dtype=np.uint64)
    y = np.arange(y0, y1, dtype=np.uint64)
    z = np.mod(np.arange(z0, z1, dtype=np.int64), N).astype(np.uint64)
    Z, Y, X = np.meshgrid(z, y, x, indexing="ij")
    n = np.uint64(N)
    return (X + n * (Y + n * Z) + np.uint64(1)).ravel()


def test_windows_independent():
    ws = [_window(p) for p in PATCHES]
    for i in range(len(ws)):
        for j in range(i):
            assert _disjoint(ws[i], ws[j]), (PATCHES[i], PATCHES[j])


@pytest.fixture(scope="module")
def ctx():
    import torch

    import dccrg_amd as D
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    c = D.Context(0, 0, 1)
    yield c
    c.close()


@pytest.mark.gpu
def test_gol_2048_cubed_patches(ctx):
    import dccrg_amd as D

    rng = np.random.default_rng(2048)
    g = (D.Dccrg().set_initial_length((N, N, N)).set_neighborhood_length(1)
         .set_maximum_refinement_level(0).set_periodic(False, False, True).initialize(ctx))
    try:
        assert g.n_local == N ** 3
        for f in ("a", "b", "n"):
            g.add_field(f, np.uint32)  # zero-initialised (dccrg.hpp:7153-7184 value-initialises)
        expect = []
        for p in PATCHES:
            w = _window(p)
            dims = tuple(hi - lo for lo, hi in w)
            box = np.zeros(dims[::-1], dtype=np.uint32)  # [z, y, x]
            ox, oy, oz = p[0] - w[0][0], p[1] - w[1][0], p[2] - w[2][0]
            box[oz:oz + P, oy:oy + P, ox:ox + P] = rng.random((P, P, P)) < 0.2
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
        # nothing outside the windows is alive or has a live neighbor
        assert g.checksum(cur) == tuple(sa)
        assert g.checksum("n") == tuple(sn)
    finally:
        g.close()
