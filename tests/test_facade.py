"""The C++ drop-in facade (include/dccrg_amd.hpp): user programs written the
way the reference's examples use dccrg::Dccrg, compiled against the facade
with the reference's own flags (-std=c++11, Makefile:8) and run on the GPU,
also as several MPI ranks sharing the GPU (mpiexec -n 3, as the reference's
.tstN targets run); results compared with the oracle."""
import os
import subprocess

import numpy as np
import pytest

from oracle import dccrg_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "facade_programs")
MPI_INC, MPI_LIB = "/opt/conda/include", "/opt/conda/lib"


def compile_facade(out=BIN):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["g++", "-std=c++11", "-pedantic", "-Werror", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"), "-I", MPI_INC,
           os.path.join(ROOT, "tests", "cpp", "facade_programs.cpp"), "-o", out,
           os.path.join(ROOT, "dccrg_amd", "libdccrgx.so"), os.path.join(MPI_LIB, "libmpi.so"),
           f"-Wl,-rpath,{os.path.join(ROOT, 'dccrg_amd')}:{MPI_LIB}"]
    subprocess.check_call(cmd)
    return out


@pytest.mark.skipif(not os.path.exists(os.path.join(MPI_INC, "mpi.h")), reason="MPI headers absent")
def test_facade_compiles(tmp_path):
    compile_facade(str(tmp_path / "facade_programs"))


@pytest.mark.skipif(not os.path.exists(os.path.join(MPI_INC, "mpi.h")), reason="MPI headers absent")
def test_derived_datatype_flattening(tmp_path):
    """detail::flatten (the facade packs derived cell datatypes by memcpy of
    their byte blocks) equals MPI_Pack / MPI_Unpack for every constructor:
    vector, hvector, indexed, hindexed, indexed_block, struct with padding,
    resized, dup, nesting, absolute addresses, pair types with gaps."""
    out = str(tmp_path / "flatten_check")
    subprocess.check_call(["g++", "-std=c++11", "-pedantic", "-Werror", "-O2", "-Wall", "-I",
                           os.path.join(ROOT, "include"), "-I", MPI_INC,
                           os.path.join(ROOT, "tests", "cpp", "flatten_check.cpp"), "-o", out,
                           os.path.join(ROOT, "dccrg_amd", "libdccrgx.so"), os.path.join(MPI_LIB, "libmpi.so"),
                           f"-Wl,-rpath,{os.path.join(ROOT, 'dccrg_amd')}:{MPI_LIB}"])
    env = dict(os.environ, LD_LIBRARY_PATH="/usr/lib/x86_64-linux-gnu:" + MPI_LIB)
    r = subprocess.run([out], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "MISMATCH" not in r.stdout, r.stdout + r.stderr
    assert r.stdout.count(" ok ") == 13, r.stdout


def run(*args, ranks=1):
    srcs = [os.path.join(ROOT, "tests", "cpp", "facade_programs.cpp"), os.path.join(ROOT, "include", "dccrg_amd.hpp"),
            os.path.join(ROOT, "include", "dccrgx.h")]
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(os.path.getmtime(f) for f in srcs):
        compile_facade()
    env = dict(os.environ)
    env["LD_LIBRARY_PATH"] = "/usr/lib/x86_64-linux-gnu:" + MPI_LIB
    cmd = [BIN, *[str(a) for a in args]]
    if ranks > 1:  # the reference's .tstN targets: mpiexec -n 3 on one host
        cmd = [MPIEXEC, "-n", str(ranks)] + cmd
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


MPIEXEC = "/opt/conda/bin/mpiexec"


@pytest.mark.gpu
def test_facade_blinker():
    assert "PASS blinker" in run("blinker")


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [1, 3])
def test_facade_halo(ranks):
    """examples/basic_cell_data.cpp: every neighbor's copy equals its id, on
    1 rank and on 3 ranks sharing the GPU (halo over MPI through the host)."""
    out = run("halo", ranks=ranks)
    assert out.count("PASS halo") == ranks


@pytest.mark.gpu
def test_facade_mapping_matches_oracle():
    om = O.Mapping((100, 200, 300), 13)
    for line in run("mapping").strip().splitlines():
        v = [int(x) for x in line.split()]
        cid = v[0]
        assert v[1] == om.get_refinement_level(cid)
        assert tuple(v[2:5]) == om.get_indices(cid)
        assert v[5] == om.get_parent(cid) and v[6] == om.get_level_0_parent(cid)
        assert v[7] == om.get_cell_length_in_indices(cid)


def _alive_counts(out):
    got = {}
    for line in out.strip().splitlines():
        if line.startswith("alive "):
            _, cid, cnt = line.split()
            got[int(cid)] = int(cnt)
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [1, 3])
@pytest.mark.parametrize("dims,per", [((12, 10, 9), (0, 0, 1)), ((9, 7, 1), (1, 1, 0)), ((20, 6, 5), (1, 1, 1))])
def test_facade_overlap_loop(dims, per, ranks):
    """examples/game_of_life.cpp:117-139 with set_send_single_cells(true):
    start receives, start sends, inner counts, wait receives, outer counts,
    inner rules, wait sends, outer rules; get_neighbors_of_at_offset is
    checked inside the program."""
    steps = 6
    got = _alive_counts(run("overlap", *dims, steps, *per, ranks=ranks))
    n = int(np.prod(dims))
    a0 = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 200)
    ra, rc = O.gol_reference_run(dims, tuple(bool(p) for p in per), 1, a0, steps)
    assert got == {int(i) + 1: int(rc[i]) for i in np.nonzero(ra)[0]}


@pytest.mark.gpu
@pytest.mark.parametrize("dims,per", [((12, 10, 9), (0, 0, 1)), ((9, 7, 1), (1, 1, 0))])
def test_facade_scalability_loop(dims, per):
    steps = 5
    out = run("scal3d", *dims, steps, *per)
    got = {}
    for line in out.strip().splitlines():
        _, cid, cnt = line.split()
        got[int(cid)] = int(cnt)
    n = int(np.prod(dims))
    a0 = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 200)
    ra, rc = O.gol_reference_run(dims, tuple(bool(p) for p in per), 1, a0, steps)
    want = {int(i) + 1: int(rc[i]) for i in np.nonzero(ra)[0]}
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("dims,per,hood", [((4, 3, 2), (1, 0, 1), 1), ((3, 1, 1), (1, 0, 0), 2),
                                           ((5, 4, 1), (0, 0, 0), 0)])
def test_facade_iteration_cache_order(dims, per, hood):
    """neighbors_of = [only_of][both], neighbors_to = [both][only_to] (dccrg.hpp:11570-11712)."""
    og = O.Grid(dims, 0, tuple(bool(p) for p in per), hood)
    for line in run("lists", *dims, *per, hood).strip().splitlines():
        head, rest = line.split(" of", 1)
        cid = int(head.split()[1])
        of_part, to_part = rest.split(" to", 1)

        def parse(s):
            out = []
            for tok in s.split():
                i, o = tok.split(":")
                out.append((int(i), tuple(int(x) for x in o.split(","))))
            return out
        lof, lto = O.iteration_cache_lists(og.find_neighbors_of(cid), og.find_neighbors_to(cid))
        assert parse(of_part) == lof
        assert parse(to_part) == lto


@pytest.mark.gpu
def test_facade_amr_matches_oracle():
    """refine_completely / stop_refining / unrefine_completely through the
    facade: new cells and the rebuilt iteration-cache lists equal the
    oracle's, data moves as execute_refines moves it (checked in the
    program), and unrefining restores the parents."""
    from oracle.dccrg_amr import AmrOracle
    asked = [33, 8]
    o = AmrOracle((6, 5, 4), 1, (False, True, True), 1, 1)
    for c in asked:
        assert o.refine_completely(0, c)
    want_new = sorted(o.stop_refining()[0])
    out = run("amr", *asked)
    assert "PASS amr" in out, out
    lines = out.strip().splitlines()
    assert [int(x) for x in lines[0].split()[1:]] == want_new
    og = o.grid
    n_cells = 0
    for line in lines[1:]:
        if not line.startswith("cell "):
            continue
        n_cells += 1
        head, rest = line.split(" of", 1)
        cid = int(head.split()[1])
        of_part, to_part = rest.split(" to", 1)

        def parse(s):
            out = []
            for tok in s.split():
                i, off = tok.split(":")
                out.append((int(i), tuple(int(x) for x in off.split(","))))
            return out
        lof, lto = O.iteration_cache_lists(og.find_neighbors_of(cid), og.find_neighbors_to(cid))
        assert parse(of_part) == lof, cid
        assert parse(to_part) == lto, cid
    assert n_cells == len(o.cells())


@pytest.mark.gpu
def test_facade_restart(tmp_path):
    """save_grid_data / load_grid_data through the facade: the resumed game
    equals the uninterrupted one (checked in the program), and the file is
    the reference layout: header = step, No_Geometry, one u32 is_alive per
    cell (the cell's get_mpi_datatype()), cells ascending."""
    import struct
    from oracle import dccrg_checkpoint as K
    path = str(tmp_path / "gol_5.dc")
    out = run("restart", path)
    assert "PASS restart 225" in out, out
    buf = open(path, "rb").read()
    got = K.read_grid_data(buf, 0, 8)
    assert struct.unpack("<Q", got["header"])[0] == 5
    assert got["length"] == (15, 15, 1) and got["geometry"] == K.no_geometry()
    assert got["order"] == list(range(1, 226))
    assert all(len(b) == 4 and struct.unpack("<I", b)[0] in (0, 1) for b in got["cells"].values())


@pytest.mark.gpu
@pytest.mark.parametrize("dims,per,hood", [((3, 1, 1), (0, 0, 0), 1), ((4, 3, 2), (1, 0, 1), 1),
                                           ((1, 1, 1), (0, 0, 0), 1), ((5, 4, 1), (0, 0, 0), 0)])
def test_facade_get_cells_criteria(dims, per, hood):
    """get_cells(criteria, exact_match, hood) picks local cells by their
    neighbor types (is_neighbor_type_match, dccrg.hpp:2968-3075): exact =
    type mask equal to a criterion, inexact = mask AND the OR of them > 0;
    one process, so every neighbor is local and no cell is on a boundary."""
    pers = tuple(bool(p) for p in per)
    grids = {0: O.Grid(dims, 0, pers, hood)}
    n = int(np.prod(dims))
    got, faces = {}, {}
    for line in run("cells", *dims, *per, hood).strip().splitlines():
        head, _, ids = line.partition(":")
        if head.startswith("face "):
            faces[int(head.split()[1])] = [(int(a), int(b)) for a, b in (t.split("/") for t in ids.split())]
        else:
            got[head.strip()] = [int(x) for x in ids.split()]
    # get_face_neighbors_of (dccrg.hpp:2828-2955) of every cell
    for cid in range(1, n + 1):
        assert faces[cid] == [(int(i), int(d)) for i, d in grids[0].face_neighbors_of(cid)], cid
    for h, items in ((0, None), (7, [(1, 0, 0)])):
        g = grids[0]
        types = {}
        for cid in range(1, n + 1):
            t = 0
            if any(c for c, _ in g.find_neighbors_of(cid, items)):
                t |= 1
            if any(c for c in g.find_neighbors_to(cid, None if items is None else O.neighborhood_to(items))):
                t |= 2
            types[cid] = t
        assert got[f"hood {h} all"] == list(range(1, n + 1))
        for c in (0, 1, 2, 3, 4, 12):
            for exact in (0, 1):
                want = [cid for cid in range(1, n + 1) if (types[cid] == c if exact else types[cid] & c)]
                assert got[f"hood {h} crit {c} exact {exact}"] == want, (h, c, exact)


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [1, 3])
def test_facade_coordinate_lookups(ranks):
    """get_existing_cell / refine_completely_at / dont_unrefine_at over the
    Cartesian geometry (periodic wrap, end face, non-periodic miss, after a
    refinement) and get_remote_neighbors_to against the neighbor lists."""
    out = run("coords", ranks=ranks)
    assert out.count("coords ok") == ranks, out


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [1, 3])
def test_facade_converting_copy(ranks):
    """tests/constructors/copy.cpp: a grid copied into another cell type (and
    then another geometry) has the original's cells, owners, neighbor lists,
    user neighborhoods and weights, default data, and its own working remote
    neighbor updates."""
    out = run("copy", ranks=ranks)
    assert out.count("copy ok") == ranks, out


@pytest.mark.gpu
@pytest.mark.parametrize("ranks,shape", [(1, (3, 1)), (3, (3, 1)), (3, (7, 5))])
def test_facade_variable_neighbour_data(ranks, shape):
    """tests/variable_data_size/variable_neighbour_data.cpp:82-130 through the
    facade: per-cell vectors whose datatype is a struct of two addresses,
    remote copies sized by the receiver, then new sizes and one vector."""
    out = run("varneigh", *shape, ranks=ranks)
    assert out.count("varneigh ok") == ranks, out
    if ranks == 3 and shape == (3, 1):  # one cell per rank: every neighbor is remote
        assert sum(int(l.split()[-1]) for l in out.splitlines() if "varneigh ok" in l) == 4


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [1, 3])
def test_facade_user_neighborhood_game_of_life(ranks):
    """tests/user_neighborhood/game_of_life.cpp: four interlaced games over
    the user neighborhood {-2, 0, 2}^2 minus the origin (hood length 2,
    periodic 18 x 18), updated and iterated per neighborhood; the live cells
    every 4 steps are the test's known answer (glider included)."""
    out = run("interlaced", ranks=ranks)
    lines = [l for l in out.splitlines() if "interlaced ok" in l]
    assert len(lines) == ranks, out
    assert sum(int(l.split()[-1]) for l in lines) == 9 * 18 * 18  # steps 0, 4, ..., 32


def interlaced_live(gs, step):
    """The live cells of user_neighborhood/game_of_life.cpp's known answer at
    a step divisible by 4 (as tests/cpp/facade_programs.cpp states it)."""
    t, b, h, c, k = 12 * gs + 6, 14 * gs + 1, 10 * gs + 7, 15 * gs + 6, 5 * gs + 2
    r = {t, t + 2, t + 4, t + 2 + 2 * gs, t + 4 + 2 * gs, t + 6 + 2 * gs, b, b + 2, b + 4,
         h + 2, h + 4, h - 2 * gs, h - 2 * gs + 6, h - 4 * gs + 2, h - 4 * gs + 4,
         c, c + 2, c - 2 * gs, c + 6 - 4 * gs, c + 4 - 6 * gs, c + 6 - 6 * gs, k, k + 2, k - 2 * gs, k + 2 - 2 * gs}
    q = step // 4
    for x, y in [(3, 15), (5, 13), (1, 11), (3, 11), (5, 11)]:
        r.add(((y - 2 * q) % gs) * gs + (x + 2 * q) % gs)
    return r


def test_interlaced_known_answer():
    """The known answer the GPU facade test checks against, pinned by an
    independent numpy run of the same game (periodic rolls over the +-2
    neighborhood)."""
    gs = 18
    a = np.zeros((gs, gs), dtype=np.int64)  # [y, x]; id = y * gs + x + 1
    for cid in interlaced_live(gs, 0):
        a[(cid - 1) // gs, (cid - 1) % gs] = 1
    for step in range(36):
        if step % 4 == 0:
            ys, xs = np.nonzero(a)
            assert {int(y * gs + x + 1) for y, x in zip(ys, xs)} == interlaced_live(gs, step), step
        n = sum(np.roll(np.roll(a, dy, 0), dx, 1) for dy in (-2, 0, 2) for dx in (-2, 0, 2) if dy or dx)
        a = np.where(n == 3, 1, np.where(n == 2, a, 0))


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [1, 3])
def test_facade_additional_items_and_no_geometry(ranks):
    """tests/additional_cell_data/{test1,test2,neighbor_data1,neighbor_data2}.cpp:
    additional cell / neighbor items with defaults or filled in by update()
    (ids, No_Geometry centers), through grid.cells, local_cells() and
    neighbors_of, again after balance_load; zero-byte cells; No_Geometry's
    arithmetic (dccrg_no_geometry.hpp)."""
    out = run("items", ranks=ranks)
    assert out.count("items ok") == ranks, out


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [1, 3])
def test_facade_cell_data_never_copied(ranks):
    """tests/constructors/simple.cpp: a cell type whose copy / move
    constructors and assignments throw survives initialization, remote copies,
    halo updates and balance_load."""
    out = run("nocopy", ranks=ranks)
    assert out.count("nocopy ok") == ranks, out


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [1, 3])
def test_facade_write_vtk_file(ranks, tmp_path):
    """dccrg.hpp:3320-3390: each rank's file lists its leaves in ascending
    id order, 8 corners per cell (x fastest, C++ default float formatting),
    9 ints per CELLS line and voxel types; written after a refinement and the
    no-LB initialize / continue / finish_balance_load sequence."""
    out = run("vtk", str(tmp_path / "grid"), ranks=ranks)
    leaves = {}
    for line in out.splitlines():
        if line.startswith("leaf "):
            f = line.split()
            leaves.setdefault(int(f[1]), []).append((int(f[2]), [float(v) for v in f[3:]]))
    assert sum(len(v) for v in leaves.values()) == 6 - 1 + 8
    for r in range(ranks):
        cells = sorted(leaves.get(r, []))
        n = len(cells)
        want = ["# vtk DataFile Version 2.0", "Cartesian cell refinable grid", "ASCII", "DATASET UNSTRUCTURED_GRID",
                f"POINTS {n * 8} float"]
        for _, (x0, y0, z0, x1, y1, z1) in cells:
            for k in range(8):
                want.append(" ".join("%g" % v for v in (x1 if k & 1 else x0, y1 if k & 2 else y0, z1 if k & 4 else z0)))
        want.append(f"CELLS {n} {n * 9}")
        want += ["8 " + "".join(f"{j * 8 + i} " for i in range(8)) for j in range(n)]
        want.append(f"CELL_TYPES {n}")
        want += ["11"] * n
        assert (tmp_path / f"grid_{r}.vtk").read_text().split("\n")[:-1] == want, r
