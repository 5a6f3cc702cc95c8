"""Grid data files from device fields (dccrgx_save_grid_data /
dccrgx_grid_load / dccrgx_load_cell_data) against the oracle's restatement
of the reference layout (oracle/dccrg_checkpoint.py, dccrg.hpp:1109-2427):
written bytes identical to the oracle's for the same cell order; files in
any cell order and from any writer rank count load into the right cells;
tests/restart's round trips (game of life resumed from a file, the
variable-size two-pass load of variable_cell_data.cpp)."""
import struct

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from oracle import dccrg_checkpoint as K  # noqa: E402
from oracle import dccrg_oracle as O  # noqa: E402
from test_gpu_explicit import leaves_for  # noqa: E402

GEOM = K.cartesian_geometry((0.0, 0.0, 0.0), (1 / 15, 1 / 15, 1 / 15))


def make(length, M, per, hood, P, leaves=None):
    out = []
    for r in range(P):
        c = D.Context(0, r, P)
        g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
             .set_neighborhood_length(hood).initialize(c, leaves=leaves))
        g._keep = c
        out.append(g)
    return out


def fill(g):
    """u32 a = id % 1000, f64 b = id / 7, u8 c = id % 251 (a 13-byte record)."""
    ids = g.local_cells()
    g.add_field("a", np.uint32)
    g.add_field("b", np.float64)
    g.add_field("c", np.uint8)
    g.write_local("a", (ids % 1000).astype(np.uint32))
    g.write_local("b", ids.astype(np.float64) / 7)
    g.write_local("c", (ids % 251).astype(np.uint8))


def record(cid):
    return struct.pack("<IdB", cid % 1000, cid / 7, cid % 251)


def save_all(grids, path, fields, offset=0, header=b"", geometry=GEOM):
    sizes = [g.save_sizes(fields) for g in grids]
    for g in grids:
        g.save_grid_data(path, offset, header, fields, geometry, all_sizes=sizes)


CASES = [  # length, M, periodic, hood, leaves spec
    ((6, 5, 4), 0, (True, False, True), 1, None),
    ((9, 7, 1), 2, (True, True, False), 0, None),
    ((4, 3, 2), 2, (False, False, False), 0, 20),
    ((3, 4, 3), 1, (True, False, False), 1, 30),
]


def leaves_of(case):
    length, M, per, hood, nref = case
    return None if nref is None else leaves_for((length, M, per, hood, nref, 3))


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("case", CASES)
def test_saved_bytes_match_oracle(tmp_path, case, P):
    length, M, per, hood, _ = case
    grids = make(length, M, per, hood, P, leaves_of(case))
    for g in grids:
        fill(g)
    path = str(tmp_path / "g.dc")
    hdr = struct.pack("<Q", 25)
    save_all(grids, path, ["a", "b", "c"], offset=8, header=hdr)
    ranks = [[(int(c), record(int(c))) for c in g.local_cells()] for g in grids]
    want = K.write_grid_data(8, hdr, length, grids[0].info.max_ref_lvl, hood, per, GEOM, ranks,
                             prefix=b"\0" * 8)
    assert open(path, "rb").read() == want


@pytest.mark.parametrize("writers,readers", [(1, 1), (3, 1), (1, 2), (2, 3)])
@pytest.mark.parametrize("case", CASES)
def test_load_any_rank_count(tmp_path, case, writers, readers):
    """Saved on `writers` ranks, loaded on `readers` ranks: every cell's
    data arrives (cell_overlaps_local, dccrg.hpp:2059-2071)."""
    length, M, per, hood, _ = case
    grids = make(length, M, per, hood, writers, leaves_of(case))
    for g in grids:
        fill(g)
    path = str(tmp_path / "g.dc")
    save_all(grids, path, ["a", "b", "c"])
    seen = []
    for r in range(readers):
        c = D.Context(0, r, readers)
        g, hdr, geo = D.Dccrg.start_loading_grid_data(c, path)
        assert geo == GEOM and g._length == tuple(length) and g._periodic == tuple(per)
        g.add_field("a", np.uint32)
        g.add_field("b", np.float64)
        g.add_field("c", np.uint8)
        g.continue_loading_grid_data(["a", "b", "c"])
        g.finish_loading_grid_data()
        ids = g.local_cells()
        assert np.array_equal(g.read_local("a"), (ids % 1000).astype(np.uint32))
        assert np.array_equal(g.read_local("b"), ids.astype(np.float64) / 7)
        assert np.array_equal(g.read_local("c"), (ids % 251).astype(np.uint8))
        seen += [int(x) for x in ids]
        g.close()
        c.close()
    assert sorted(seen) == sorted(int(x) for g in grids for x in g.local_cells())


@pytest.mark.parametrize("writers,readers", [(2, 3), (3, 1)])
@pytest.mark.parametrize("case", CASES[:2] + CASES[3:])
def test_sfc_grid_round_trip(tmp_path, case, writers, readers):
    """A file saved by an SFC-placed grid loads into an SFC-placed grid on
    another rank count: each reader holds exactly the cells the SFC
    placement gives it (same table as a fresh SFC grid, sfc.hip), with their
    data."""
    length, M, per, hood, _ = case
    leaves = leaves_of(case)
    grids = []
    for r in range(writers):
        c = D.Context(0, r, writers)
        g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
             .set_neighborhood_length(hood).set_initial_partition("sfc").initialize(c, leaves=leaves))
        g._keep = c
        fill(g)
        grids.append(g)
    path = str(tmp_path / "g.dc")
    save_all(grids, path, ["a", "b", "c"])
    seen = []
    for r in range(readers):
        c = D.Context(0, r, readers)
        g, _, _ = D.Dccrg.start_loading_grid_data(c, path, partition="sfc")
        fresh = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
                 .set_neighborhood_length(hood).set_initial_partition("sfc").initialize(c, leaves=leaves))
        ids = g.local_cells()
        assert np.array_equal(ids, fresh.local_cells())
        fresh.close()
        for f, t in (("a", np.uint32), ("b", np.float64), ("c", np.uint8)):
            g.add_field(f, t)
        g.continue_loading_grid_data(["a", "b", "c"])
        g.finish_loading_grid_data()
        assert np.array_equal(g.read_local("a"), (ids % 1000).astype(np.uint32))
        assert np.array_equal(g.read_local("b"), ids.astype(np.float64) / 7)
        seen += [int(x) for x in ids]
        g.close()
        c.close()
    assert sorted(seen) == sorted(int(x) for g in grids for x in g.local_cells())


@pytest.mark.parametrize("case", CASES[:3])
def test_load_shuffled_oracle_file(tmp_path, case):
    """A file whose cells are listed in a random order, split over 4 writer
    ranks (the reference writes get_cells() order, a hash order), read in two
    passes: first the u32 member, then the rest (continue_loading_grid_data
    advances every cell's offset)."""
    length, M, per, hood, _ = case
    (g0,) = make(length, M, per, hood, 1, leaves_of(case))
    cells = [int(c) for c in g0.local_cells()]
    g0.close()
    rng = np.random.default_rng(5)
    order = [cells[i] for i in rng.permutation(len(cells))]
    cuts = np.sort(rng.integers(0, len(order) + 1, 3))
    parts = np.split(np.array(order), cuts)
    ranks = [[(int(c), record(int(c))) for c in p] for p in parts]
    path = str(tmp_path / "o.dc")
    open(path, "wb").write(K.write_grid_data(0, b"abc", length, M, hood, per, K.no_geometry(), ranks))
    ctx = D.Context(0, 0, 1)
    g, hdr, geo = D.Dccrg.start_loading_grid_data(ctx, path, 0, 3)
    assert hdr == b"abc" and geo == K.no_geometry()
    assert [int(c) for c in g.local_cells()] == sorted(cells)
    g.add_field("a", np.uint32)
    g.add_field("b", np.float64)
    g.add_field("c", np.uint8)
    g.continue_loading_grid_data(["a"])
    g.continue_loading_grid_data(["b", "c"])
    g.finish_loading_grid_data()
    ids = g.local_cells()
    assert np.array_equal(g.read_local("a"), (ids % 1000).astype(np.uint32))
    assert np.array_equal(g.read_local("b"), ids.astype(np.float64) / 7)
    assert np.array_equal(g.read_local("c"), (ids % 251).astype(np.uint8))
    g.close()
    ctx.close()


@pytest.mark.parametrize("L,per", [((40, 24, 16), (True, False, True)), ((64, 48, 1), (True, True, False))])
def test_game_of_life_restart(tmp_path, L, per):
    """tests/restart/restart_test.cpp's property: a game resumed from a file
    (the step in the header) continues exactly as the uninterrupted one."""
    n = int(np.prod(L))
    a0 = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 250)
    ref_a, ref_n = O.gol_reference_run(L, per, 1, a0, 10)
    ctx = D.Context(0, 0, 1)
    g = D.Dccrg().set_initial_length(L).set_periodic(*per).set_neighborhood_length(1).initialize(ctx)
    for f in ("a", "b", "n"):
        g.add_field(f, np.uint32)
    g.write_local("a", a0)
    cur, nxt = "a", "b"
    for _ in range(4):
        g.gol_step(cur, nxt, "n")
        cur, nxt = nxt, cur
    path = str(tmp_path / "gol_4.dc")
    g.save_grid_data(path, 0, struct.pack("<Q", 4), [cur, "n"])
    g.close()
    g, hdr, _ = D.Dccrg.start_loading_grid_data(ctx, path, 0, 8)
    assert struct.unpack("<Q", hdr)[0] == 4
    for f in ("a", "b", "n"):
        g.add_field(f, np.uint32)
    g.continue_loading_grid_data(["a", "n"])
    g.finish_loading_grid_data()
    cur, nxt = "a", "b"
    for _ in range(6):
        g.gol_step(cur, nxt, "n")
        cur, nxt = nxt, cur
    assert np.array_equal(g.read_local(cur), ref_a)
    assert np.array_equal(g.read_local("n"), ref_n)
    g.close()
    ctx.close()


@pytest.mark.parametrize("writers,readers", [(1, 1), (3, 2)])
def test_variable_cell_data_restart(tmp_path, writers, readers):
    """tests/restart/variable_cell_data.cpp: 20x1x1; cell c (c % 4 != 0)
    holds ints 0..c-1 and data_size = c.  Saved as (u64 data_size, ints);
    loaded in two passes: the sizes, then (after resizing) the ints."""
    grids = make((20, 1, 1), 0, (False, False, False), 1, writers)
    for g in grids:
        g.add_field("size", np.uint64)
        g.add_variable_field("data", np.int32)
        ids = [int(c) for c in g.local_cells()]
        cnt = [c if c % 4 else 0 for c in ids]
        g.write_local("size", np.array(cnt, dtype=np.uint64))
        g.resize("data", ids, cnt)
        g.write_cells("data", ids, [np.arange(k, dtype=np.int32) for k in cnt])
    path = str(tmp_path / "variable_cell_data.dc")
    save_all(grids, path, ["size", "data"], geometry=K.cartesian_geometry((0, 0, 0), (1, 1, 1)))
    ranks = [[(int(c), struct.pack("<Q", c if c % 4 else 0) + np.arange(c if c % 4 else 0, dtype=np.int32).tobytes())
              for c in (int(x) for x in g.local_cells())] for g in grids]
    assert open(path, "rb").read() == K.write_grid_data(0, b"", (20, 1, 1), 0, 1, (False, False, False),
                                                        K.cartesian_geometry((0, 0, 0), (1, 1, 1)), ranks)
    for r in range(readers):
        c = D.Context(0, r, readers)
        g, _, _ = D.Dccrg.start_loading_grid_data(c, path)
        g.add_field("size", np.uint64)
        g.add_variable_field("data", np.int32)
        g.continue_loading_grid_data(["size"])
        ids = [int(x) for x in g.local_cells()]
        sizes = g.read_local("size")
        assert sizes.tolist() == [x if x % 4 else 0 for x in ids]
        g.resize("data", ids, sizes.astype(np.uint32))
        g.continue_loading_grid_data(["data"])
        g.finish_loading_grid_data()
        for cid, arr in zip(ids, g.read_cells("data", ids)):
            assert arr.tolist() == list(range(cid if cid % 4 else 0))
        g.close()
        c.close()


def test_large_uniform_round_trip(tmp_path):
    """256^3 cells, two u32 fields (128 MiB of records): the contiguous fast
    path both ways, and loading only the first member of each record."""
    L = (256, 256, 256)
    ctx = D.Context(0, 0, 1)
    g = D.Dccrg().set_initial_length(L).set_neighborhood_length(1).initialize(ctx)
    g.add_field("a", np.uint32)
    g.add_field("b", np.uint32)
    D.lib().dccrgx_field_init_hash(g._h, g.field_id("a"), 500)
    D.lib().dccrgx_field_init_hash(g._h, g.field_id("b"), 100)
    a, b = g.read_local("a"), g.read_local("b")
    path = str(tmp_path / "big.dc")
    g.save_grid_data(path, 0, b"", ["a", "b"])
    g.close()
    g, _, _ = D.Dccrg.start_loading_grid_data(ctx, path)
    assert g.info.uniform == 1
    g.add_field("a", np.uint32)
    g.add_field("b", np.uint32)
    g.continue_loading_grid_data(["a", "b"])
    assert np.array_equal(g.read_local("a"), a) and np.array_equal(g.read_local("b"), b)
    g.close()
    g, _, _ = D.Dccrg.start_loading_grid_data(ctx, path)
    g.add_field("a", np.uint32)
    g.continue_loading_grid_data(["a"])
    assert np.array_equal(g.read_local("a"), a)
    g.close()
    ctx.close()


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("case", CASES)
def test_reference_reader_parses_device_files(tmp_path, P, case):
    """A device-written file (header u64 time step, u64 is_alive per cell, as
    tests/restart writes) parsed by the reference's own reader
    (tests/restart/dc2vtk.cpp built where it lies, oracle/_ref)."""
    import ref_reader as R
    if not R.available():
        pytest.skip("oracle/_ref/restart_dc2vtk is built where the reference is")
    length, M, per, hood, _ = case
    grids = make(length, M, per, hood, P, leaves_of(case))
    start, l0 = (0.5, -1.0, 2.0), (0.25, 0.5, 0.125)
    order = []
    for g in grids:
        ids = g.local_cells()
        order += ids.tolist()
        g.add_field("alive", np.uint64)
        g.write_local("alive", (ids % 3 == 0).astype(np.uint64))
    path = str(tmp_path / "dev.dc")
    save_all(grids, path, ["alive"], 0, struct.pack("<Q", 9), K.cartesian_geometry(start, l0))
    pts, alive = R.read_with_reference(path)
    assert alive.tolist() == [int(c % 3 == 0) for c in order]
    np.testing.assert_allclose(pts, R.expected_corners(order, length, grids[0].get_maximum_refinement_level(),
                                                       start, l0), rtol=1e-5, atol=1e-9)
    for g in grids:
        g.close()
