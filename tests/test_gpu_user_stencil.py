"""Device user stencils (include/dccrgx_stencil.hpp): user functors run by
for_each_cell over a region's cells see every cell once, with its id and
slot, and walk its neighbors_of in the reference's iteration-cache order
(dccrg.hpp:11590-11640: unique (id, offset) pairs, the ones whose id is not
also a neighbor_to first, each group ascending by (id, x, y, z)).

The functors are examples/user_stencil.hip (built by build()):
- us_digest: per cell an order-sensitive digest of its (neighbor id, x, y, z)
  sequence, neighbor ids read from a field whose ghosts were exchanged;
  checked against the oracle's find_neighbors_of / find_neighbors_to lists
  (oracle/dccrg_oracle.c) grouped as the iteration cache groups them
  (oracle iteration_cache_lists);
- us_gol: examples/game_of_life.cpp:54-79 as a functor, inner then outer
  region, checked against live-neighbor counts over the same lists.
Uniform grids (neighbors in closed form, the wrap-aware key selection near
periodic boundaries: 1- and 2-cell periodic axes give self and duplicate ids)
and grids with refined cells (stencil rows regrouped), one and three ranks
(loopback halos), the default and an asymmetric user neighborhood."""
import ctypes as C
import os

import numpy as np
import pytest

from oracle import dccrg_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "examples", "libuser_stencil.so")
M64 = (1 << 64) - 1
K1, K2, K3, PR = 0x100000001B3, 0x5851F42D4C957F2D, 0x14057B7EF767814F, 0x100000001B3
# not symmetric (only-neighbors_of entries exist), within the grid's neighborhood length
USER_ITEMS = {1: [[-1, 0, 1], [1, 1, 1], [0, -1, 0], [1, -1, 0], [0, 0, -1]],
              2: [[-2, 0, 1], [1, 1, 1], [0, -1, 0], [2, -2, 2]]}

CASES = [  # length, periodic, hood length, max level, refined level-0 cells
    ((10, 8, 6), (False, False, False), 1, 0, 0),
    ((10, 8, 6), (True, True, True), 1, 0, 0),
    ((12, 5, 1), (True, False, False), 2, 0, 0),
    ((1, 1, 1), (True, True, True), 1, 0, 0),
    ((2, 3, 2), (True, True, True), 1, 0, 0),
    ((6, 5, 4), (True, True, False), 1, 1, 40),
    ((6, 5, 4), (False, True, True), 1, 1, 30),
    ((5, 4, 3), (True, True, True), 2, 1, 10),
]


def lib():
    L = C.CDLL(LIB)
    L.us_gol.argtypes = [C.c_void_p] + [C.c_int32] * 5
    L.us_digest.argtypes = [C.c_void_p] + [C.c_int32] * 6
    L.us_region_cells.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
    L.us_region_cells.restype = C.c_longlong
    L.us_gol_staged.argtypes = [C.c_void_p] + [C.c_int32] * 6
    L.us_digest_staged.argtypes = [C.c_void_p] + [C.c_int32] * 6
    L.us_fsum_staged.argtypes = [C.c_void_p] + [C.c_int32] * 6
    L.us_fsum32_staged.argtypes = [C.c_void_p] + [C.c_int32] * 6
    return L


def test_example_library_exports():
    """CPU: build() made the user-stencil program and it exports its entry points."""
    L = C.CDLL(LIB)
    for s in ("us_gol", "us_digest", "us_region_cells", "us_gol_staged", "us_digest_staged", "us_fsum_staged",
              "us_fsum32_staged"):
        assert hasattr(L, s)


def digest(entries, mix):
    h = 0xCBF29CE484222325
    for i, (x, y, z) in entries:
        v = (mix[i] + x * K1 + y * K2 + z * K3) & M64
        h = ((h ^ v) * PR) & M64
    return h


def refined(length, n_ref, seed):
    rng = np.random.default_rng(seed)
    m = O.Mapping(length, 1)
    n0 = int(np.prod(length))
    ref = set(int(v) for v in rng.choice(np.arange(1, n0 + 1), size=n_ref, replace=False))
    leaves = []
    for c in range(1, n0 + 1):
        leaves += m.get_all_children(c) if c in ref else [c]
    return sorted(leaves)


@pytest.mark.gpu
@pytest.mark.parametrize("user_hood", [False, True])
@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("case", CASES)
def test_user_stencil_iteration_order(case, P, user_hood):
    import torch

    import dccrg_amd as D
    from dccrg_amd import _capi as X
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    length, per, hood_len, M, n_ref = case
    leaves = refined(length, n_ref, 7) if n_ref else None
    all_cells = leaves if leaves else list(range(1, int(np.prod(length)) + 1))
    og = O.Grid(length, M, per, hood_len, all_cells)
    hood = 5 if user_hood else D.DEFAULT_NEIGHBORHOOD_ID
    items = np.array(USER_ITEMS[hood_len], dtype=np.int32)
    lists = {}
    for c in all_cells:
        if user_hood:
            nof, nto = og.find_neighbors_of(c, items), og.find_neighbors_to(c, -items)
        else:
            nof, nto = og.find_neighbors_of(c), og.find_neighbors_to(c)
        lists[c] = O.iteration_cache_lists(nof, nto)[0]
    ids = np.array(all_cells, dtype=np.uint64)
    mix = dict(zip(all_cells, (int(v) for v in O.splitmix64(ids))))
    alive = dict(zip(all_cells, (int(v) for v in O.random_alive(ids, 400))))
    L = lib()
    ctxs, grids = [], []
    for r in range(P):
        ctx = D.Context(0, r, P)
        g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
             .set_neighborhood_length(hood_len).initialize(ctx, leaves=leaves))
        if user_hood:
            assert g.add_neighborhood(hood, USER_ITEMS[hood_len])
        for f, t in (("id", np.uint64), ("cid", np.uint64), ("dig", np.uint64), ("cnt", np.uint32),
                     ("a", np.uint32), ("b", np.uint32), ("n", np.uint32), ("scid", np.uint64),
                     ("sdig", np.uint64), ("scnt", np.uint32), ("sb", np.uint32), ("sn", np.uint32)):
            g.add_field(f, t)
        loc = g.local_cells()
        g.write_local("id", loc)
        g.write_local("a", np.array([alive[int(c)] for c in loc], dtype=np.uint32))
        g.write_local("b", np.full(loc.size, 0xFFFFFFFF, dtype=np.uint32))
        ctxs.append(ctx)
        grids.append(g)
    try:
        # ghosts of the ids and the alive state, then the functors
        msgs = {}
        for r, g in enumerate(grids):
            for p in g.get_cells_to_send(hood):
                buf = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                msgs[(r, p)] = (buf, g.pack_to(p, buf.data_ptr(), buf.numel(), hood=hood, fields=["id", "a"]))
                g.ctx.synchronize()
        for r, g in enumerate(grids):
            g.halo_self(hood=hood, fields=["id", "a"])
            for p in g.get_cells_to_receive(hood):
                buf, nb = msgs[(p, r)]
                g.unpack_from(p, buf.data_ptr(), nb, hood=hood, fields=["id", "a"])
            g.ctx.synchronize()
        for g in grids:
            fid = g.field_id
            h = g._h
            n_in = L.us_region_cells(h, hood, X.REGION_INNER)
            n_out = L.us_region_cells(h, hood, X.REGION_OUTER)
            assert n_in + n_out == g.n_local == L.us_region_cells(h, hood, X.REGION_ALL)
            assert g.stencil_view(hood).n_cells == g.n_local
            loc = [int(c) for c in g.local_cells()]
            g.write_local("cid", np.zeros(len(loc), dtype=np.uint64))
            assert L.us_digest(h, hood, X.REGION_INNER, fid("id"), fid("cid"), fid("dig"), fid("cnt")) == 0
            g.ctx.synchronize()
            inner = set(int(c) for c in g.read_local("cid") if c)
            assert len(inner) == n_in
            if n_ref:  # refined grids: the reference's inner cells
                assert inner == set(int(c) for c in g.inner_cells(hood))
            else:  # uniform: whole slices whose cells read no ghost copy
                local = set(loc)
                assert all(i in local for c in inner for i, _ in lists[c])
            assert L.us_digest(h, hood, X.REGION_OUTER, fid("id"), fid("cid"), fid("dig"), fid("cnt")) == 0
            for region in (X.REGION_INNER, X.REGION_OUTER):
                assert L.us_gol(h, hood, fid("a"), fid("b"), fid("n"), region) == 0
                # the staged launches: values instead of slots (the staged
                # kernel where the neighborhood is the cube or the faces)
                assert L.us_gol_staged(h, hood, fid("a"), fid("sb"), fid("sn"), region, 1) == 0
                assert L.us_digest_staged(h, hood, region, fid("id"), fid("scid"), fid("sdig"), fid("scnt")) == 0
            g.ctx.synchronize()
            assert g.read_local("cid").tolist() == loc
            assert g.read_local("scid").tolist() == loc
            for pre in ("", "s"):
                got_cnt = g.read_local(pre + "cnt").tolist()
                got_dig = g.read_local(pre + "dig").tolist()
                got_n = g.read_local(pre + "n").tolist()
                got_b = g.read_local(pre + "b").tolist()
                for k, c in enumerate(loc):
                    want = lists[c]
                    assert got_cnt[k] == len(want), (pre, c, got_cnt[k], want)
                    assert got_dig[k] == digest(want, mix), (pre, c, want)
                    n = sum(alive[i] for i, _ in want)
                    assert got_n[k] == n, (pre, c)
                    assert got_b[k] == (1 if n == 3 else (alive[c] if n == 2 else 0)), (pre, c)
    finally:
        for g in grids:
            g.close()
        for ctx in ctxs:
            ctx.close()


@pytest.mark.gpu
def test_user_stencil_view_follows_refinement():
    """The view's data is remade after a structural change: refine, then the
    functor's digests follow the new leaves."""
    import torch

    import dccrg_amd as D
    from dccrg_amd import _capi as X
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    length, per = (4, 4, 3), (True, False, True)
    ctx = D.Context(0, 0, 1)
    g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(1).set_periodic(*per)
         .set_neighborhood_length(1).initialize(ctx))
    L = lib()
    try:
        for f, t in (("id", np.uint64), ("cid", np.uint64), ("dig", np.uint64), ("cnt", np.uint32)):
            g.add_field(f, t)
        for step in range(2):
            loc = [int(c) for c in g.local_cells()]
            g.write_local("id", np.array(loc, dtype=np.uint64))
            h = g._h
            assert L.us_digest(h, D.DEFAULT_NEIGHBORHOOD_ID, X.REGION_ALL, g.field_id("id"), g.field_id("cid"),
                               g.field_id("dig"), g.field_id("cnt")) == 0
            ctx.synchronize()
            og = O.Grid(length, 1, per, 1, loc)
            mix = dict(zip(loc, (int(v) for v in O.splitmix64(np.array(loc, dtype=np.uint64)))))
            dig = g.read_local("dig").tolist()
            for k, c in enumerate(loc):
                want = O.iteration_cache_lists(og.find_neighbors_of(c), og.find_neighbors_to(c))[0]
                assert dig[k] == digest(want, mix), (step, c)
            if step == 0:
                for c in (6, 23, 40):
                    g.refine_completely(c)
                g.stop_refining()
    finally:
        g.close()
        ctx.close()


LARGER = [((70, 40, 9), (True, False, True), 1),
          ((66, 36, 11), (False, True, False), 2),
          ((130, 33, 5), (True, True, True), 1),
          # A % 4 == 0 (16-byte staged loads), several tiles along A and B
          ((132, 37, 12), (False, True, True), 1),
          ((128, 50, 7), (True, True, False), 0),
          ((8, 20, 16), (True, False, False), 1),
          # A and B not periodic, A % 4 == 0: the staged kernel takes the
          # boundary columns and rows too (the edge walk none of the ring)
          ((68, 29, 10), (False, False, True), 1),
          ((64, 40, 9), (False, False, False), 0),
          ((136, 18, 7), (False, True, False), 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("staged", [None, 0, 1, 2, 3])
@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("length,per,hood_len", LARGER)
def test_gol_functor_larger_grids(length, per, hood_len, P, staged):
    """The game-of-life functor over several steps on grids where most cells
    take the fixed-distance walk (no boundary within reach), with wraps and
    rank slabs: equal to the oracle's run (oracle gol_reference_run, the
    reference's lists) on every rank.  staged: None = for_each_cell (slots),
    1 = for_each_cell_staged (the staged kernel for the cube / faces plus the
    boundary walks on a second stream), 2 = the same on the caller's stream
    alone, 3 = 1 with one workgroup per tile marching through every slice
    (long marches: every plane after the second fetched while two are in
    flight), 0 = for_each_cell_staged with every cell walked."""
    import torch

    import dccrg_amd as D
    from dccrg_amd import _capi as X
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    n = int(np.prod(length))
    ids = np.arange(1, n + 1, dtype=np.uint64)
    a0 = O.random_alive(ids, 300)
    steps = 3
    ref_a, ref_n = O.gol_reference_run(length, per, hood_len, a0, steps)
    L = lib()
    hood = D.DEFAULT_NEIGHBORHOOD_ID
    ctxs, grids = [], []
    for r in range(P):
        ctx = D.Context(0, r, P)
        g = (D.Dccrg().set_initial_length(length).set_periodic(*per).set_neighborhood_length(hood_len)
             .initialize(ctx))
        for f in ("a", "b", "n"):
            g.add_field(f, np.uint32)
        g.write_local("a", a0[g.local_cells().astype(np.int64) - 1])
        ctxs.append(ctx)
        grids.append(g)
    try:
        cur, nxt = "a", "b"
        for _ in range(steps):
            msgs = {}
            for r, g in enumerate(grids):
                for p in g.get_cells_to_send():
                    buf = torch.empty(1 << 22, dtype=torch.uint8, device="cuda")
                    torch.cuda.synchronize()
                    msgs[(r, p)] = (buf, g.pack_to(p, buf.data_ptr(), buf.numel(), fields=[cur]))
                    g.ctx.synchronize()
            for r, g in enumerate(grids):
                g.halo_self(fields=[cur])
                for p in g.get_cells_to_receive():
                    buf, nb = msgs[(p, r)]
                    g.unpack_from(p, buf.data_ptr(), nb, fields=[cur])
                g.ctx.synchronize()
            for g in grids:
                if staged is None:
                    assert L.us_gol(g._h, hood, g.field_id(cur), g.field_id(nxt), g.field_id("n"),
                                    X.REGION_ALL) == 0
                else:
                    for region in (X.REGION_INNER, X.REGION_OUTER):
                        assert L.us_gol_staged(g._h, hood, g.field_id(cur), g.field_id(nxt), g.field_id("n"),
                                               region, staged) == 0
                g.ctx.synchronize()
            cur, nxt = nxt, cur
        for g in grids:
            idx = g.local_cells().astype(np.int64) - 1
            assert np.array_equal(g.read_local(cur), ref_a[idx])
            assert np.array_equal(g.read_local("n"), ref_n[idx])
    finally:
        for g in grids:
            g.close()
        for ctx in ctxs:
            ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("length,per,hood_len", [((68, 40, 9), (True, False, True), 1),
                                                 ((33, 20, 14), (False, True, True), 1),
                                                 ((64, 18, 10), (True, True, True), 0),
                                                 ((20, 16, 12), (True, False, True), 2)])
def test_staged_f64_order(length, per, hood_len, P):
    """A floating-point functor over two staged f64 fields, summed over the
    neighbors in order (us_fsum_staged): the staged launch gives the same
    bits as the walk (same neighbors, same order), and both are within
    1e-12 of the sum in the reference's iteration order over the oracle's
    lists (fp64 contraction may differ from numpy)."""
    import torch

    import dccrg_amd as D
    from dccrg_amd import _capi as X
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    n = int(np.prod(length))
    ids = np.arange(1, n + 1, dtype=np.uint64)
    rng = np.random.default_rng(11)
    u0, w0 = rng.standard_normal(n), rng.uniform(0.5, 1.5, n)
    og = O.Grid(length, 0, per, hood_len, list(range(1, n + 1)))
    L = lib()
    hood = D.DEFAULT_NEIGHBORHOOD_ID
    ctxs, grids = [], []
    for r in range(P):
        ctx = D.Context(0, r, P)
        g = (D.Dccrg().set_initial_length(length).set_periodic(*per).set_neighborhood_length(hood_len)
             .initialize(ctx))
        for f in ("u", "w", "o1", "o0"):
            g.add_field(f, np.float64)
        idx = g.local_cells().astype(np.int64) - 1
        g.write_local("u", u0[idx])
        g.write_local("w", w0[idx])
        ctxs.append(ctx)
        grids.append(g)
    try:
        msgs = {}
        for r, g in enumerate(grids):
            for p in g.get_cells_to_send():
                buf = torch.empty(1 << 22, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                msgs[(r, p)] = (buf, g.pack_to(p, buf.data_ptr(), buf.numel(), fields=["u", "w"]))
                g.ctx.synchronize()
        for r, g in enumerate(grids):
            g.halo_self(fields=["u", "w"])
            for p in g.get_cells_to_receive():
                buf, nb = msgs[(p, r)]
                g.unpack_from(p, buf.data_ptr(), nb, fields=["u", "w"])
            g.ctx.synchronize()
        for g in grids:
            f = g.field_id
            for region in (X.REGION_INNER, X.REGION_OUTER):
                assert L.us_fsum_staged(g._h, hood, f("u"), f("w"), f("o1"), region, 1) == 0
                assert L.us_fsum_staged(g._h, hood, f("u"), f("w"), f("o0"), region, 0) == 0
            g.ctx.synchronize()
            got1, got0 = g.read_local("o1"), g.read_local("o0")
            assert np.array_equal(got1.view(np.uint64), got0.view(np.uint64))
            loc = g.local_cells()
            want = np.empty(loc.size)
            for k, c in enumerate(loc):
                c = int(c)
                me = u0[c - 1]
                s = me
                for i, _ in O.iteration_cache_lists(og.find_neighbors_of(c), og.find_neighbors_to(c))[0]:
                    s += w0[i - 1] * u0[i - 1] - 0.25 * me
                want[k] = s
            assert np.allclose(got1, want, rtol=1e-12, atol=1e-12)
    finally:
        for g in grids:
            g.close()
        for ctx in ctxs:
            ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("staged", [1, 3])
@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("length,per,hood_len", [((68, 29, 10), (False, False, True), 1),
                                                 ((64, 40, 9), (False, False, False), 0),
                                                 ((132, 37, 12), (False, True, True), 1),
                                                 ((72, 20, 8), (True, False, True), 1)])
def test_staged_f32_two_fields(length, per, hood_len, P, staged):
    """Two staged f32 fields (the LDS-DMA kernel with two fields, its edge
    columns and the row march; staged 3: long marches): the staged launch
    gives the same bits as the walk, and both are within 1e-4 of a float64
    sum in the reference's iteration order over the oracle's lists."""
    import torch

    import dccrg_amd as D
    from dccrg_amd import _capi as X
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    n = int(np.prod(length))
    rng = np.random.default_rng(12)
    u0 = rng.standard_normal(n).astype(np.float32)
    w0 = rng.uniform(0.5, 1.5, n).astype(np.float32)
    og = O.Grid(length, 0, per, hood_len, list(range(1, n + 1)))
    L = lib()
    hood = D.DEFAULT_NEIGHBORHOOD_ID
    ctxs, grids = [], []
    for r in range(P):
        ctx = D.Context(0, r, P)
        ctxs.append(ctx)
        g = (D.Dccrg().set_initial_length(length).set_periodic(*per).set_neighborhood_length(hood_len)
             .initialize(ctx))
        for f in ("u", "w", "o1", "o0"):
            g.add_field(f, np.float32)
        idx = g.local_cells().astype(np.int64) - 1
        g.write_local("u", u0[idx])
        g.write_local("w", w0[idx])
        grids.append(g)
    try:
        msgs = {}
        for r, g in enumerate(grids):
            for p in g.get_cells_to_send():
                buf = torch.empty(1 << 22, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                msgs[(r, p)] = (buf, g.pack_to(p, buf.data_ptr(), buf.numel(), fields=["u", "w"]))
                g.ctx.synchronize()
        for r, g in enumerate(grids):
            g.halo_self(fields=["u", "w"])
            for p in g.get_cells_to_receive():
                buf, nb = msgs[(p, r)]
                g.unpack_from(p, buf.data_ptr(), nb, fields=["u", "w"])
            g.ctx.synchronize()
        for g in grids:
            f = g.field_id
            for region in (X.REGION_INNER, X.REGION_OUTER):
                assert L.us_fsum32_staged(g._h, hood, f("u"), f("w"), f("o1"), region, staged) == 0
                assert L.us_fsum32_staged(g._h, hood, f("u"), f("w"), f("o0"), region, 0) == 0
            g.ctx.synchronize()
            got1, got0 = g.read_local("o1"), g.read_local("o0")
            assert np.array_equal(got1.view(np.uint32), got0.view(np.uint32))
            loc = g.local_cells()
            want = np.empty(loc.size)
            for k, c in enumerate(loc):
                c = int(c)
                me = float(u0[c - 1])
                s = me
                for i, _ in O.iteration_cache_lists(og.find_neighbors_of(c), og.find_neighbors_to(c))[0]:
                    s += float(w0[i - 1]) * float(u0[i - 1]) - 0.25 * me
                want[k] = s
            assert np.allclose(got1.astype(np.float64), want, rtol=1e-4, atol=1e-4)
    finally:
        for g in grids:
            g.close()
        for ctx in ctxs:
            ctx.close()
