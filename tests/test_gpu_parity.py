"""GPU parity: libdccrgx.so (HIP, gfx950) against the CPU oracle and the
reference's own known answers.  Integer results must match bit for bit.

Several ranks are emulated in ONE process on one GPU (one context per rank,
halo messages moved with the transport-free pack/unpack entry points); the
RCCL transport itself is exercised by bench.py at N > 1.
"""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from dccrg_amd import _capi as X  # noqa: E402
from oracle import dccrg_oracle as O  # noqa: E402

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    c = D.Context(0, 0, 1)
    yield c
    c.close()


def make_grid(length, periodic, hood, max_ref_lvl=0, rank=0, size=1):
    c = D.Context(0, rank, size)
    g = (D.Dccrg().set_initial_length(length).set_periodic(*periodic)
         .set_neighborhood_length(hood).set_maximum_refinement_level(max_ref_lvl).initialize(c))
    g._ctx_keep = c
    return g


# ---------------------------------------------------------------- mapping ----
MAP_CASES = [((10, 10, 1), 0), ((3, 3, 1), 1), ((400, 400, 1), 2), ((100, 200, 300), 13),
             ((2048, 2048, 2048), 0), ((2048, 2048, 2048), 10), ((1, 1, 1), 20), ((7, 13, 11), 5)]


@pytest.mark.parametrize("length,lvl", MAP_CASES)
def test_mapping_bit_exact(ctx, length, lvl):
    om = O.Mapping(length, lvl)
    dm = D.Mapping(length, lvl)
    assert dm.last_cell == om.last_cell
    rng = np.random.default_rng(1234 + lvl)
    last = om.last_cell
    ids = np.concatenate([
        rng.integers(0, last + 2, size=20000, dtype=np.uint64),
        np.array([0, 1, last, last + 1, 2**64 - 1], dtype=np.uint64),
    ])
    # level boundaries
    n0 = length[0] * length[1] * length[2]
    first = 1
    for l in range(lvl + 1):
        ids = np.concatenate([ids, np.array([first - 1, first, first + 1], dtype=np.uint64)])
        first += n0 * 8**l
    ids = ids[ids <= np.uint64(2**64 - 1)]
    ref_idx, ref_lvl = om.ids_to_indices(ids)
    t = torch.from_numpy(ids.view(np.int64)).to(DEV)
    idx, lv = dm.ids_to_indices(t)
    torch.cuda.synchronize()
    assert np.array_equal(lv.cpu().numpy(), ref_lvl)
    assert np.array_equal(idx.cpu().numpy().view(np.uint64), ref_idx)
    # inverse on valid cells, plus random indices / levels (incl. invalid)
    ok = ref_lvl >= 0
    back = dm.indices_to_ids(idx[torch.from_numpy(ok).to(DEV)], lv[torch.from_numpy(ok).to(DEV)])
    torch.cuda.synchronize()
    assert np.array_equal(back.cpu().numpy().view(np.uint64), ids[ok])
    G = np.array(length, dtype=np.uint64) * np.uint64(2**lvl)
    ridx = np.stack([rng.integers(0, int(g) + 2, size=5000, dtype=np.uint64) for g in G], axis=1)
    rlvl = rng.integers(-1, lvl + 2, size=5000).astype(np.int32)
    want = om.indices_to_ids(ridx, rlvl)
    got = dm.indices_to_ids(torch.from_numpy(ridx.view(np.int64)).to(DEV),
                            torch.from_numpy(rlvl).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)
    # octree relations
    sample = ids[:3000]
    ts = torch.from_numpy(sample.view(np.int64)).to(DEV)
    for op, f in [(X.OP_LENGTH_IN_INDICES, om.get_cell_length_in_indices),
                  (X.OP_PARENT, om.get_parent), (X.OP_LEVEL_0_PARENT, om.get_level_0_parent),
                  (X.OP_CHILD, om.get_child)]:
        got = dm.ids_op(op, ts).cpu().numpy().view(np.uint64)
        want = np.array([f(int(c)) for c in sample[:600]], dtype=np.uint64)
        assert np.array_equal(got[:600], want), op


@pytest.mark.parametrize("n", [1, 255, 511, 512, 513, 1024, 5000, (1 << 21) + 7])
def test_mapping_kernel_bit_exact(ctx, n):
    """The batched get_indices kernel (two ids per lane per pass, LDS-staged
    stores), with partial last passes, against the oracle."""
    length, lvl = (2048, 2048, 2048), 10
    om = O.Mapping(length, lvl)
    dm = D.Mapping(length, lvl)
    rng = np.random.default_rng(n)
    ids = rng.integers(0, om.last_cell + 2, size=n, dtype=np.uint64)
    ref_idx, ref_lvl = om.ids_to_indices(ids)
    idx, lv = dm.ids_to_indices(torch.from_numpy(ids.view(np.int64)).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(lv.cpu().numpy(), ref_lvl)
    assert np.array_equal(idx.cpu().numpy().view(np.uint64), ref_idx)


# ------------------------------------------------------- neighbor lists ----
NBR_CASES = [
    ((10, 10, 1), (False, False, False), 1, 0),
    ((3, 2, 1), (True, False, False), 1, 0),
    ((3, 2, 1), (True, False, False), 1, 1),
    ((3, 1, 1), (True, False, False), 2, 0),
    ((4, 4, 4), (True, True, True), 1, 0),
    ((4, 4, 4), (True, True, True), 2, 0),
    ((5, 3, 4), (False, True, False), 0, 2),
    ((1, 1, 1), (True, True, True), 1, 0),
    ((2, 1, 3), (True, True, True), 3, 1),
    ((6, 5, 1), (True, True, True), 1, 0),
]


@pytest.mark.parametrize("length,periodic,hood,lvl", NBR_CASES)
def test_neighbor_lists_match_oracle(length, periodic, hood, lvl):
    og = O.Grid(length, lvl, periodic, hood)
    g = make_grid(length, periodic, hood, lvl)
    cells = og.cells()
    row, ids, off = g.neighbors_of(cells)
    for i, c in enumerate(cells):
        want = og.find_neighbors_of(int(c))
        got = [(int(ids[k]), tuple(int(v) for v in off[k])) for k in range(int(row[i]), int(row[i + 1]))]
        assert got == want, (int(c), got, want)
    row, ids = g.neighbors_to(cells)
    for i, c in enumerate(cells):
        want = og.find_neighbors_to(int(c))
        got = [int(v) for v in ids[int(row[i]):int(row[i + 1])]]
        assert got == want, int(c)


# ---------------------------------------------- classification + lists ----
RANK_CASES = [
    ((10, 10, 1), (False, False, False), 1, 3),
    ((10, 10, 1), (True, True, False), 1, 4),
    ((6, 5, 4), (False, False, True), 1, 2),
    ((6, 5, 4), (True, True, True), 2, 3),
    ((5, 4, 3), (False, False, False), 0, 5),
    ((7, 13, 11), (True, True, True), 2, 3),
    ((2, 2, 2), (True, True, True), 1, 8),
    ((3, 3, 1), (False, False, False), 1, 12),  # more ranks than cells
]


@pytest.mark.parametrize("length,periodic,hood", [
    ((128, 128, 80), (False, False, False), 1),
    ((96, 64, 40), (True, False, True), 2),
    ((3000, 7, 1), (False, True, False), 1),
    ((40, 30, 20), (True, True, False), 3),   # 342 items: the per-cell fill path
])
def test_neighbor_lists_many_cells(length, periodic, hood):
    """Row pointers of every cell (device scan over many tiles) against the
    closed-form count, the entries of a random sample against the oracle."""
    og = O.Grid(length, 0, periodic, hood)
    g = make_grid(length, periodic, hood, 0)
    n = int(np.prod(length))
    cells = np.arange(1, n + 1, dtype=np.uint64)
    row, ids, off = g.neighbors_of(cells)
    lin = np.arange(n)
    pos = [lin % length[0], (lin // length[0]) % length[1], lin // (length[0] * length[1])]
    cnt = np.ones(n, dtype=np.int64)
    for d in range(3):
        valid = np.zeros(n, dtype=np.int64)
        for o in range(-hood, hood + 1):
            valid += 1 if periodic[d] else ((pos[d] + o >= 0) & (pos[d] + o < length[d]))
        cnt *= valid
    cnt -= 1
    assert row[0] == 0 and np.array_equal(np.diff(row.astype(np.int64)), cnt)
    rng = np.random.default_rng(3)
    for c in rng.choice(cells, size=400, replace=False):
        i = int(c) - 1
        got = [(int(ids[k]), tuple(int(v) for v in off[k])) for k in range(int(row[i]), int(row[i + 1]))]
        assert got == og.find_neighbors_of(int(c)), int(c)
    g.close()


def block_owner_np(total, P, ids):
    """dccrg.hpp:8098-8145 vectorised (the oracle's block_owner)."""
    cpp = 1 if total < P else total // P + (1 if total % P else 0)
    fewer = cpp * P - total
    i = ids.astype(np.int64) - 1
    split = fewer * (cpp - 1)
    return np.where(i < split, i // max(cpp - 1, 1), fewer + (i - split) // cpp)


@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("periodic", [(False, False, False), (True, False, True)])
def test_rank_lists_100_cubed(P, periodic):
    """every rank's per-peer send / receive lists of the
    100^3 block partition (slabs that end mid-plane), hood 1, against a
    vectorised restatement of dccrg.hpp:8729-8891 (uniform hood 1 is
    symmetric, so neighbors_to = neighbors_of as sets)."""
    L = (100, 100, 100)
    n = int(np.prod(L))
    ids = np.arange(1, n + 1, dtype=np.int64)
    x, y, z = (ids - 1) % L[0], ((ids - 1) // L[0]) % L[1], (ids - 1) // (L[0] * L[1])
    own = block_owner_np(n, P, ids)
    pairs = []
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if not (dx or dy or dz):
                    continue
                c = [x + dx, y + dy, z + dz]
                ok = np.ones(n, dtype=bool)
                for d in range(3):
                    if periodic[d]:
                        c[d] = c[d] % L[d]
                    else:
                        ok &= (c[d] >= 0) & (c[d] < L[d])
                nid = c[0] + L[0] * (c[1] + L[1] * c[2]) + 1
                pairs.append((ids[ok], nid[ok]))
    cell = np.concatenate([p[0] for p in pairs])
    nbr = np.concatenate([p[1] for p in pairs])
    oc, on = own[cell - 1], own[nbr - 1]
    for r in range(P):
        g = make_grid(L, periodic, 1, 0, r, P)
        m = (oc == r) & (on != r)
        want_recv = {int(p): np.unique(nbr[m & (on == p)]).tolist() for p in np.unique(on[m])}
        want_send = {int(p): np.unique(cell[m & (on == p)]).tolist() for p in np.unique(on[m])}
        assert g.get_cells_to_receive() == want_recv, r
        assert g.get_cells_to_send() == want_send, r
        assert g.get_number_of_update_send_cells() == sum(len(v) for v in want_send.values())
        outer = np.unique(cell[m])
        assert np.array_equal(g.outer_cells(), outer.astype(np.uint64)), r
        g.close()


@pytest.mark.parametrize("length,periodic,hood,P", RANK_CASES)
def test_rank_structures_match_oracle(length, periodic, hood, P):
    og = O.Grid(length, 0, periodic, hood)
    for r in range(P):
        ref = og.rank_view(r, P)
        g = make_grid(length, periodic, hood, 0, r, P)
        assert g.local_cells().tolist() == ref["local"]
        assert g.outer_cells().tolist() == ref["outer"]
        assert g.inner_cells().tolist() == ref["inner"]
        assert g.remote_cells().tolist() == ref["remote"]
        assert g.get_cells_to_send() == ref["send"]
        assert g.get_cells_to_receive() == ref["recv"]
        assert g.get_number_of_update_send_cells() == sum(len(v) for v in ref["send"].values())
        assert g.get_number_of_update_receive_cells() == sum(len(v) for v in ref["recv"].values())
        assert g.get_number_of_update_send_cells(12345) == (1 << 64) - 1  # dccrg.hpp:5454-5456
        g.close()


# ----------------------------------------------------------------- halo ----
def loopback_halo(grids, fields):
    """Move every rank's messages to their peers through device buffers."""
    msgs = {}
    for r, g in enumerate(grids):
        for p in g.get_cells_to_send():
            buf = torch.empty(1 << 22, dtype=torch.uint8, device=DEV)
            torch.cuda.synchronize()
            n = g.pack_to(p, buf.data_ptr(), buf.numel(), fields=fields)
            g.ctx.synchronize()
            msgs[(r, p)] = (buf, n)
    for r, g in enumerate(grids):
        g.halo_self(fields=fields)
        for p in g.get_cells_to_receive():
            buf, n = msgs[(p, r)]
            g.unpack_from(p, buf.data_ptr(), n, fields=fields)
        g.ctx.synchronize()


@pytest.mark.parametrize("length,periodic,hood,P", RANK_CASES[:6])
def test_halo_ghosts_are_ids(length, periodic, hood, P):
    """examples/basic_cell_data.cpp:27-53: data = id; after the update every
    neighbor's copy equals its id."""
    grids = [make_grid(length, periodic, hood, 0, r, P) for r in range(P)]
    for g in grids:
        g.add_field("id", np.uint64)
        g.add_field("half", np.uint32)
        g.write_local("id", g.local_cells())
        g.write_local("half", (g.local_cells() // 2).astype(np.uint32))
    loopback_halo(grids, ["id", "half"])
    for g in grids:
        rem = g.remote_cells()
        recv = set(c for v in g.get_cells_to_receive().values() for c in v)
        got = g.read_remote("id")
        half = g.read_remote("half")
        for c, v, h in zip(rem, got, half):
            if int(c) in recv:
                assert int(v) == int(c) and int(h) == int(c) // 2


def test_basic_cell_data_kat():
    k = GOLD["halo_kat"]
    test_halo_ghosts_are_ids(tuple(k["length"]), tuple(bool(p) for p in k["periodic"]),
                             k["hood_length"], 3)


# ------------------------------------------------------------ game of life --
def gol_gpu(length, periodic, hood, alive0, steps, P=1, mode="step"):
    """Run the device stencil; alive0 indexed by id-1.  Returns (alive, count)."""
    grids = [make_grid(length, periodic, hood, 0, r, P) for r in range(P)]
    for g in grids:
        for f in ("a", "b", "n"):
            g.add_field(f, np.uint32)
        loc = g.local_cells().astype(np.int64)
        g.write_local("a", alive0[loc - 1])
    cur, nxt = "a", "b"
    for _ in range(steps):
        if P == 1 and mode == "step":
            grids[0].gol_step(cur, nxt, "n")
        else:
            loopback_halo(grids, [cur])
            for g in grids:
                if mode == "split":
                    g.gol_compute(cur, nxt, "n", X.REGION_INNER)
                    g.gol_compute(cur, nxt, "n", X.REGION_OUTER)
                else:
                    g.gol_compute(cur, nxt, "n", X.REGION_ALL)
        cur, nxt = nxt, cur
    n = int(np.prod(length))
    alive = np.zeros(n, dtype=np.uint32)
    count = np.zeros(n, dtype=np.uint32)
    for g in grids:
        loc = g.local_cells().astype(np.int64)
        alive[loc - 1] = g.read_local(cur)
        count[loc - 1] = g.read_local("n")
    return alive, count


GOL_CASES = [
    ((15, 15, 1), (False, False, False), 1, 1),
    ((64, 48, 1), (True, True, False), 1, 1),
    ((64, 48, 1), (True, True, True), 1, 1),
    ((70, 1, 1), (True, False, False), 1, 1),
    ((1, 70, 1), (False, True, True), 1, 1),
    ((33, 20, 17), (False, False, False), 1, 1),
    ((33, 20, 17), (True, True, True), 1, 1),
    ((65, 17, 9), (True, False, True), 1, 3),
    ((16, 16, 16), (True, True, True), 2, 2),
    ((16, 12, 10), (False, True, False), 0, 4),
    ((20, 20, 1), (True, True, False), 1, 3),
    ((9, 9, 9), (True, True, True), 1, 5),
    ((2, 3, 2), (True, True, True), 1, 1),
]


@pytest.mark.parametrize("length,periodic,hood,P", GOL_CASES)
def test_gol_bit_exact(length, periodic, hood, P):
    n = int(np.prod(length))
    ids = np.arange(1, n + 1, dtype=np.uint64)
    a0 = O.random_alive(ids, 300)
    steps = 6
    ref_a, ref_n = O.gol_reference_run(length, periodic, hood, a0, steps)
    for mode in (("step",) if P == 1 else ("all", "split")):
        a, c = gol_gpu(length, periodic, hood, a0, steps, P, mode)
        assert np.array_equal(a, ref_a), mode
        assert np.array_equal(c, ref_n), mode


VEC_CASES = [
    ((12, 20, 9), (True, True, True), 1),
    ((264, 20, 5), (False, False, False), 1),
    ((8, 40, 6), (True, False, True), 3),
    ((520, 33, 4), (True, True, False), 2),
    ((4, 4, 7), (False, True, True), 1),
    ((264, 20, 1), (True, False, False), 1),   # 2-D: vectorised row kernel
    ((1032, 9, 1), (False, True, True), 2),
    ((8, 1, 1), (True, False, False), 1),
]


@pytest.mark.parametrize("variant", ["vector", "scalar"])
@pytest.mark.parametrize("chunk", ["0", "1", "3"])
@pytest.mark.parametrize("length,periodic,P", VEC_CASES)
def test_gol_kernels_bit_exact(lib_options, variant, chunk, length, periodic, P):
    """The 26-neighbor stencil kernels the library launches (vector tiles and
    the scalar LDS kernels) against the oracle, including partial slabs, tile
    overhangs and chunk seams (the alternative tilings are checked against the
    vector kernel by tools/gol_sweep.hip)."""
    if variant == "scalar":
        lib_options("gol_scalar", 1)
    lib_options("gol_chunk", int(chunk))
    n = int(np.prod(length))
    a0 = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 350)
    ref_a, ref_n = O.gol_reference_run(length, periodic, 1, a0, 4)
    a, c = gol_gpu(length, periodic, 1, a0, 4, P, "split" if P > 1 else "step")
    assert np.array_equal(a, ref_a) and np.array_equal(c, ref_n)


VEC2D_CASES = [
    ((264, 20, 1), (True, False, False), 1),
    ((264, 20, 1), (True, True, False), 1),
    ((1028, 37, 1), (True, True, False), 1),   # strip overhang with periodic wrap
    ((1028, 37, 1), (False, False, False), 3),
    ((1032, 9, 1), (False, True, True), 2),
    ((520, 61, 1), (True, True, True), 2),
    ((8, 1, 1), (True, False, False), 1),
    ((2048, 40, 1), (False, True, False), 4),
]


@pytest.mark.parametrize("variant", ["vector", "scalar"])
@pytest.mark.parametrize("chunk", ["0", "3", "11"])
@pytest.mark.parametrize("length,periodic,P", VEC2D_CASES)
def test_gol2d_kernels_bit_exact(lib_options, variant, chunk, length, periodic, P):
    """The 2-D (LB == 1) kernels: the vector LDS row kernel and the scalar
    row kernel, over several chunk lengths, partial slabs, strip overhangs and
    periodic wraps."""
    if variant == "scalar":
        lib_options("gol_scalar", 1)
    lib_options("gol_chunk", int(chunk))
    n = int(np.prod(length))
    a0 = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 350)
    ref_a, ref_n = O.gol_reference_run(length, periodic, 1, a0, 4)
    a, c = gol_gpu(length, periodic, 1, a0, 4, P, "split" if P > 1 else "step")
    assert np.array_equal(a, ref_a) and np.array_equal(c, ref_n)


def test_gol_kat_15x15():
    k = GOLD["gol_kat"]
    n = int(np.prod(k["length"]))
    for P in (1, 3):
        a0 = np.zeros(n, dtype=np.uint32)
        a0[np.array(k["initial_live"]) - 1] = 1
        state = a0
        for step in range(k["steps"]):
            live = set((np.nonzero(state)[0] + 1).tolist())
            assert set(k["always_alive"]) <= live, step
            assert set(k["alive_even_steps" if step % 2 == 0 else "alive_odd_steps"]) <= live
            if str(step) in k["glider"]:
                assert set(k["glider"][str(step)]) <= live
            state, _ = gol_gpu(k["length"], k["periodic"], 1, state, 1, P, "split")


def test_simple_gol_blinker():
    k = GOLD["simple_gol"]
    n = int(np.prod(k["length"]))
    a0 = np.zeros(n, dtype=np.uint32)
    a0[np.array(k["initial_live"]) - 1] = 1
    a, _ = gol_gpu(k["length"], k["periodic"], 1, a0, k["turns"], 1)
    live = set((np.nonzero(a)[0] + 1).tolist())
    # turns is even: the state after the last (odd-index) turn
    assert set(k["after_odd_turn_alive"]) <= live and not (set(k["after_odd_turn_dead"]) & live)


def test_line_kat_16384():
    """tests/game_of_life/scalability.cpp:116-213 at the C2 size (16384^2):
    after its 16 steps exactly rows y0 +- 16 are alive.  Continued to 40
    steps, every row must equal the oracle's run on a narrow periodic grid
    (the state stays invariant along x)."""
    L = (16384, 16384, 1)
    y0 = 8192
    g = make_grid(L, (True, True, False), 1)
    for f in ("a", "b", "n"):
        g.add_field(f, np.uint32)
    n = L[0] * L[1]
    a0 = np.zeros(n, dtype=np.uint32)
    a0[y0 * L[0]:(y0 + 1) * L[0]] = 1
    g.write_local("a", a0)
    cur, nxt = "a", "b"
    for step in range(1, 41):
        g.gol_step(cur, nxt, "n")
        cur, nxt = nxt, cur
        if step == GOLD["line_kat"]["steps"]:
            a = g.read_local(cur).reshape(L[1], L[0])
            assert np.nonzero(a.any(axis=1))[0].tolist() == [y0 - 16, y0 + 16]
            assert int(a.sum()) == 2 * L[0]
    a = g.read_local(cur).reshape(L[1], L[0])
    c = g.read_local("n").reshape(L[1], L[0])
    W = 8
    narrow = np.zeros(W * L[1], dtype=np.uint32)
    narrow[y0 * W:(y0 + 1) * W] = 1
    ra, rc = O.gol_reference_run((W, L[1], 1), (True, True, False), 1, narrow, 40)
    ra, rc = ra.reshape(L[1], W), rc.reshape(L[1], W)
    assert np.array_equal(a, np.tile(ra[:, :1], (1, L[0])))
    assert np.array_equal(c, np.tile(rc[:, :1], (1, L[0])))


def test_gol_3d_random_vs_oracle_64():
    L = (64, 64, 64)
    n = int(np.prod(L))
    a0 = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 200)
    ref_a, ref_n = O.gol_reference_run(L, (False, False, True), 1, a0, 3)
    a, c = gol_gpu(L, (False, False, True), 1, a0, 3, 1)
    assert np.array_equal(a, ref_a) and np.array_equal(c, ref_n)


def test_user_neighborhood_lengths():
    """tests/user_neighborhood/neighbor_list_length.cpp on the device lists."""
    k = GOLD["neighbor_list_length"]
    g = make_grid(tuple(k["length"]), (True, True, True), k["hood_length"])
    cells = np.array([1, 57, 1000], dtype=np.uint64)
    for hood in k["hoods"]:
        hid = X.DEFAULT_NEIGHBORHOOD_ID if hood["id"] is None else hood["id"]
        if hood["items"] is not None:
            assert g.add_neighborhood(hid, hood["items"])
        row, ids, off = g.neighbors_of(cells, hid)
        rt, tids = g.neighbors_to(cells, hid)
        for i in range(len(cells)):
            nof = [(int(ids[j]), tuple(int(v) for v in off[j])) for j in range(int(row[i]), int(row[i + 1]))]
            nto = [int(v) for v in tids[int(rt[i]):int(rt[i + 1])]]
            lof, lto = O.iteration_cache_lists(nof, nto)
            assert len(lof) == hood["nof"] and len(lto) == hood["nto"], hood["src"]
    for bad in k["rejected"]:
        assert not g.add_neighborhood(bad["id"], bad["items"]), bad["why"]


def test_user_neighborhood_gol_matches_oracle():
    L, per = (12, 10, 8), (True, False, True)
    items = np.array([[-2, 0, 0], [1, 1, 0], [0, -1, 1], [2, 2, -2], [0, 0, 1]], dtype=np.int32)
    og = O.Grid(L, 0, per, 2)
    n = int(np.prod(L))
    a0 = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 400)
    for P in (1, 3):
        grids = [make_grid(L, per, 2, 0, r, P) for r in range(P)]
        for r, g in enumerate(grids):
            assert g.add_neighborhood(7, items)
            ref = og.rank_view(r, P, items)
            assert g.outer_cells(7).tolist() == ref["outer"]
            assert g.get_cells_to_send(7) == ref["send"]
            assert g.get_cells_to_receive(7) == ref["recv"]
            for f in ("a", "b", "n"):
                g.add_field(f, np.uint32)
            g.write_local("a", a0[g.local_cells().astype(np.int64) - 1])
        msgs = {}
        for r, g in enumerate(grids):
            for p in g.get_cells_to_send(7):
                buf = torch.empty(1 << 20, dtype=torch.uint8, device=DEV)
                torch.cuda.synchronize()
                msgs[(r, p)] = (buf, g.pack_to(p, buf.data_ptr(), buf.numel(), 7, ["a"]))
                g.ctx.synchronize()
        for r, g in enumerate(grids):
            g.halo_self(7, ["a"])
            for p in g.get_cells_to_receive(7):
                buf, nb = msgs[(p, r)]
                g.unpack_from(p, buf.data_ptr(), nb, 7, ["a"])
            g.gol_compute("a", "b", "n", X.REGION_ALL, 7)
        # reference: count of live cells over the user neighborhood's neighbors_of
        cnt = np.zeros(n, dtype=np.uint32)
        for c in range(1, n + 1):
            cnt[c - 1] = sum(int(a0[i - 1] != 0) for i, _ in og.find_neighbors_of(c, items))
        for g in grids:
            loc = g.local_cells().astype(np.int64)
            assert np.array_equal(g.read_local("n"), cnt[loc - 1])


# ------------------------------------------------------------ empty batches ----
@pytest.mark.parametrize("refined", [False, True])
def test_empty_batches(refined):
    """Every batched entry point accepts n = 0 (null id arrays): OK, the row
    pointer array's single entry is 0, and nothing else is written."""
    import ctypes as C
    L = D.lib()
    leaves = None
    length = (4, 3, 2)
    if refined:
        m = O.Mapping(length, 1)
        leaves = sorted(set(range(1, 25)) - {5}) + m.get_all_children(5)
    c = D.Context(0, 0, 1)
    g = (D.Dccrg().set_initial_length(length).set_neighborhood_length(1).set_maximum_refinement_level(1)
         .set_periodic(True, False, False).initialize(c, leaves=leaves))
    g.add_field("x", np.uint32)
    row = torch.full((1,), 7, dtype=torch.int64, device=DEV)
    torch.cuda.synchronize()
    from dccrg_amd._capi import check as ok
    H = D.DEFAULT_NEIGHBORHOOD_ID
    ok(L.dccrgx_neighbors_of(g._h, H, None, 0, row.data_ptr(), None, None, 0, None))
    ok(L.dccrgx_neighbors_of(g._h, H, None, 0, row.data_ptr(), row.data_ptr(), row.data_ptr(), 0, None))
    ok(L.dccrgx_neighbors_to(g._h, H, None, 0, row.data_ptr(), None, 0, None))
    ok(L.dccrgx_gather_neighbors(g._h, H, g.field_id("x"), None, 0, row.data_ptr(), None, 0, None))
    ok(L.dccrgx_face_neighbors_of(g._h, None, 0, row.data_ptr(), None, None, 0, None))
    ok(L.dccrgx_slots_of(g._h, None, 0, None, None))
    ok(L.dccrgx_get_process(g._h, None, 0, None))
    mp = D.Mapping(length, 1)
    ok(L.dccrgx_map_ids_to_indices(C.byref(mp._m), None, 0, None, None, None))
    ok(L.dccrgx_map_indices_to_ids(C.byref(mp._m), None, None, 0, None, None))
    ok(L.dccrgx_map_ids_op(C.byref(mp._m), 0, None, 0, None, None))
    c.synchronize()
    assert int(row[0]) == 0
    assert g.get_all_cells().size == (24 if not refined else 31)
    g.close()
    c.close()
