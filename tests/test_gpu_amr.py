"""GPU parity of adaptive mesh refinement: the library's request calls and
stop_refining (dccrg.hpp:2456-2806, 3483-3543, 9730-10693) against the CPU
restatement oracle/dccrg_amr.py on the same request sequences -- request
return values, leaf sets, new and removed cells per rank, the rebuilt
neighbor lists and per-rank lists, and the movement of cell data."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from oracle import dccrg_oracle as O  # noqa: E402
from oracle.dccrg_amr import AmrOracle  # noqa: E402
from dccrg_amd.grid import stop_refining_all, test_option  # noqa: E402


def make_ranks(length, M, per, hood, P, leaves=None):
    grids = []
    for r in range(P):
        c = D.Context(0, r, P)
        g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
             .set_neighborhood_length(hood).initialize(c, leaves=leaves))
        g._keep = c
        grids.append(g)
    return grids


def stop_all(grids):
    reqs = [g.amr_requests() for g in grids]
    union = [np.unique(np.concatenate([r[k] for r in reqs])).astype(np.uint64) for k in range(4)]
    return stop_refining_all(grids, union)


def all_leaves(grids):
    return sorted(int(c) for g in grids for c in g.local_cells())


def check_structure(grids, o: AmrOracle):
    assert all_leaves(grids) == o.cells()
    og = o.grid
    P = len(grids)
    for r, g in enumerate(grids):
        ref = og.rank_view(r, P)
        loc = [int(c) for c in g.local_cells()]
        assert loc == ref["local"]
        assert [int(c) for c in g.inner_cells()] == ref["inner"]
        assert [int(c) for c in g.outer_cells()] == ref["outer"]
        assert [int(c) for c in g.remote_cells()] == ref["remote"]
        if loc:
            cells = np.array(loc, dtype=np.uint64)
            row, ids, off = g.neighbors_of(cells)
            for i, c in enumerate(loc):
                got = [(int(ids[k]), tuple(int(v) for v in off[k])) for k in range(int(row[i]), int(row[i + 1]))]
                assert got == og.find_neighbors_of(c), c
            row, ids = g.neighbors_to(cells)
            for i, c in enumerate(loc):
                assert [int(v) for v in ids[int(row[i]):int(row[i + 1])]] == og.find_neighbors_to(c), c
        assert g.get_cells_to_send() == ref["send"]
        assert g.get_cells_to_receive() == ref["recv"]


@pytest.mark.parametrize("P", [1, 2, 3])
def test_dont_refine_cases_on_device(P):
    """tests/refine/dont_refine.cpp's three scenarios, replayed on the device
    and on the oracle step by step."""
    scen = [
        [("dont_refine", 1), ("refine", 1), "stop"],
        [("refine", 2), "stop", ("dont_refine", 1), ("refine", 6), "stop", ("dont_refine", 1), ("refine", 7), "stop"],
        [("refine", 3), "stop", ("dont_refine", 1), ("refine", 8), "stop", ("refine", 37), "stop"],
    ]
    for steps in scen:
        o = AmrOracle((3, 1, 1), -1, hood_length=1, comm_size=P)
        grids = make_ranks((3, 1, 1), -1, (False, False, False), 1, P)
        for st in steps:
            if st == "stop":
                got = stop_all(grids)
                want = o.stop_refining()
                for r in range(P):
                    assert [int(c) for c in got[r]] == want[r]
                check_structure(grids, o)
                continue
            # every process makes the call, as in the reference test (only the
            # owner accepts a refine; dont_refine is accepted everywhere)
            kind, cell = st
            for rr in range(P):
                if kind == "refine":
                    assert grids[rr].refine_completely(cell) == o.refine_completely(rr, cell)
                else:
                    assert grids[rr].dont_refine(cell) == o.dont_refine(rr, cell)
        assert 4 not in o.leaves
        for g in grids:
            g.close()


SEQ_CASES = [  # length, M, periodic, hood, P, rounds, seed
    ((4, 3, 2), 2, (False, False, False), 1, 1, 4, 0),
    ((4, 4, 1), 2, (True, True, False), 1, 2, 4, 1),
    ((5, 3, 3), 2, (True, False, True), 1, 3, 3, 2),
    ((4, 4, 2), 2, (False, True, False), 0, 2, 4, 3),
    ((3, 3, 3), 1, (True, True, True), 2, 2, 3, 4),
    ((6, 2, 1), 3, (True, False, False), 1, 1, 5, 5),
]


@pytest.fixture(params=["full", "incremental", "incremental_full_nto", "small_walks"])
def rebuild_mode(request, lib_options):
    """The rebuild's neighbors_of: recomputed for every leaf, or copied for
    rows that reference no removed leaf (explicit.hip nof_incremental; the
    library picks it above 2^20 leaves, the test option forces it).  After
    an incremental neighbors_of one rank also updates neighbors_to around the
    changes (nto_incremental); incremental_full_nto keeps the full transpose.
    small_walks: override_unrefines walks the face graph as the reference
    does (amr_dev.hip k_ou_walk, test option ou_walk; the default is the
    equivalent window test k_ou_check) and the walk's first pass gets a
    4-entry queue, so the walks overflow into the second, full-size pass."""
    lib_options("incremental", 1 if request.param.startswith("incremental") else 0)
    if request.param == "incremental_full_nto":
        lib_options("full_nto", 1)
    # every rebuild checks the device leaf lookups against the host leaf list (several ranks: the
    # host-merged list; one rank: the list fetched from the device) (explicit.hip explicit_init)
    lib_options("check_init", 1)
    if request.param == "small_walks":
        lib_options("ou_walk", 1)
        lib_options("ou_small", 4)
    return request.param


@pytest.mark.parametrize("case", SEQ_CASES)
def test_random_request_sequences(case, rebuild_mode):
    length, M, per, hood, P, rounds, seed = case
    rng = np.random.default_rng(seed)
    o = AmrOracle(length, M, per, hood, P)
    grids = make_ranks(length, M, per, hood, P)
    for rnd in range(rounds):
        cells = o.cells()
        picks = rng.choice(cells, min(len(cells), 8), replace=False)
        for c in picks:
            c = int(c)
            r = o.owner(c)
            k = int(rng.integers(4)) if rnd > 0 else 0
            fn = ("refine_completely", "unrefine_completely", "dont_unrefine", "dont_refine")[k]
            if k == 3 and rng.integers(3):
                continue  # keep dont_refine rare
            got = getattr(grids[r], fn)(c)
            want = getattr(o, fn)(r, c)
            assert got == want, (fn, c)
        got = stop_all(grids)
        want = o.stop_refining()
        for r in range(P):
            assert [int(c) for c in got[r]] == want[r]
            assert [int(c) for c in grids[r].get_removed_cells()] == o.get_removed_cells(r)
            grids[r].clear_refined_unrefined_data()
        check_structure(grids, o)
        assert o.max_level_difference() <= 1
    for g in grids:
        g.close()


BATCH_CASES = [  # length, M, periodic, hood, P, rounds, seed
    ((6, 5, 1), 2, (True, True, False), 0, 1, 5, 10),
    ((4, 4, 3), 2, (False, True, True), 1, 2, 4, 11),
    ((5, 4, 2), 2, (True, False, False), 1, 3, 3, 12),
    ((4, 3, 3), 3, (True, True, True), 0, 1, 4, 13),
    ((3, 3, 2), 2, (False, False, False), 2, 2, 3, 14),
]
KINDS = (("refine_completely", 0), ("dont_unrefine", 3), ("unrefine_completely", 2), ("dont_refine", 1))


@pytest.mark.parametrize("case", BATCH_CASES)
def test_batched_requests_match_sequential_calls(case, rebuild_mode):
    """dccrgx_amr_request_cells on explicit grids runs each batch on the
    device (amr_dev.hip); its results and the four sets afterwards equal the
    reference's calls made one by one in the same order (the oracle), with
    whole sibling groups, repeated ids, cells of other ranks and ids that are
    not leaves in the batches; stop_refining then decides on the device."""
    length, M, per, hood, P, rounds, seed = case
    rng = np.random.default_rng(seed)
    leaves = [int(c) for c in O.random_balanced_leaves(length, M, per, hood, 12, seed)]
    o = AmrOracle(length, M, per, hood, P, leaves=leaves)
    grids = make_ranks(length, M, per, hood, P, leaves=np.array(leaves, dtype=np.uint64))
    m = O.Mapping(length, M)
    for rnd in range(rounds):
        cells = o.cells()
        for r in range(P):
            for name, kind in KINDS:
                if kind == 1 and rng.integers(2):
                    continue  # dont_refine in some rounds only
                pick = [int(c) for c in rng.choice(cells, min(len(cells), 10), replace=False)]
                extra = []
                for c in pick[:4]:  # whole sibling groups and their repeats
                    extra += [int(s) for s in m.get_siblings(c) if s] + [c]
                ids = pick + extra
                ids += [int(m.get_all_children(c)[0]) for c in pick[:2] if o.level(c) < M]  # not leaves
                ids = [i for i in ids if i] + [0]
                rng.shuffle(ids)
                got = grids[r].request_cells(kind, np.array(ids, dtype=np.uint64))
                want = [getattr(o, name)(r, c) for c in ids]
                assert [bool(x) for x in got] == want, (rnd, r, name)
            sets = grids[r].amr_requests()
            for k, ref in enumerate((o.to_refine, o.not_to_refine, o.to_unrefine, o.not_to_unrefine)):
                assert [int(c) for c in sets[k]] == sorted(ref[r]), (rnd, r, k)
        got = stop_all(grids)
        want = o.stop_refining()
        for r in range(P):
            assert [int(c) for c in got[r]] == want[r]
            assert [int(c) for c in grids[r].get_removed_cells()] == o.get_removed_cells(r)
            grids[r].clear_refined_unrefined_data()
        check_structure(grids, o)
        assert o.max_level_difference() <= 1
    for g in grids:
        g.close()


@pytest.mark.parametrize("P", [1, 2])
def test_own_requests_stop_refining(P):
    """stop_refining from each rank's own device state (sets == NULL, one
    rank) equals the union path and the oracle; with two ranks the union is
    gathered from the device sets (amr_requests)."""
    length, M, per, hood = (6, 6, 1), 2, (True, True, False), 0
    rng = np.random.default_rng(7)
    leaves = [int(c) for c in O.random_balanced_leaves(length, M, per, hood, 12, 3)]
    o = AmrOracle(length, M, per, hood, P, leaves=leaves)
    grids = make_ranks(length, M, per, hood, P, leaves=np.array(leaves, dtype=np.uint64))
    for rnd in range(4):
        cells = o.cells()
        for r in range(P):
            mine = [c for c in cells if o.owner(c) == r]
            for name, kind in KINDS[:3]:
                ids = [int(c) for c in rng.choice(mine, min(len(mine), 12), replace=False)]
                grids[r].request_cells(kind, np.array(ids, dtype=np.uint64))
                for c in ids:
                    getattr(o, name)(r, c)
        got = [grids[0].stop_refining()] if P == 1 else stop_all(grids)
        want = o.stop_refining()
        for r in range(P):
            assert [int(c) for c in got[r]] == want[r]
            grids[r].clear_refined_unrefined_data()
        check_structure(grids, o)
    for g in grids:
        g.close()


@pytest.mark.parametrize("P,fail_rank", [(1, 0), (2, 1), (3, 0)])
def test_two_phase_stop_refining_failure(P, fail_rank, monkeypatch):
    """One rank's stop_refining fails after its decisions (injected ENOMEM):
    no rank adopts a new leaf set, every rank keeps its own requests and its
    data, and the next stop_refining gives the oracle's result on all ranks
    (the reference's collective decisions, dccrg.hpp:3483-3507).  P == 1 runs
    the own-requests path (sets == NULL), P > 1 the union path."""
    length, M, per, hood = (5, 4, 2), 2, (True, False, True), 1
    rng = np.random.default_rng(11 + P)
    o = AmrOracle(length, M, per, hood, P)
    grids = make_ranks(length, M, per, hood, P)
    for g in grids:
        g.add_field("v", np.float64)
        g.write_local("v", g.local_cells().astype(np.float64))
    for rnd in range(3):
        cells = o.cells()
        for r in range(P):
            mine = [c for c in cells if o.owner(c) == r]
            ids = [int(c) for c in rng.choice(mine, min(len(mine), 5), replace=False)]
            name, kind = KINDS[0] if rnd == 0 else KINDS[int(rng.integers(3))]
            grids[r].request_cells(kind, np.array(ids, dtype=np.uint64))
            for c in ids:
                getattr(o, name)(r, c)
        before = [[int(c) for c in g.local_cells()] for g in grids]
        reqs = [[a.tolist() for a in g.amr_requests()] for g in grids]
        with test_option("fail_stop_refining", fail_rank + 1), pytest.raises(D.DccrgxError, match="injected"):
            if P == 1:
                grids[0].stop_refining()
            else:
                stop_all(grids)
        for r, g in enumerate(grids):
            assert [int(c) for c in g.local_cells()] == before[r]
            assert [a.tolist() for a in g.amr_requests()] == reqs[r]
            assert np.array_equal(g.read_local("v"), g.local_cells().astype(np.float64))
        got = [grids[0].stop_refining()] if P == 1 else stop_all(grids)
        want = o.stop_refining()
        for r in range(P):
            assert [int(c) for c in got[r]] == want[r]
            grids[r].clear_refined_unrefined_data()
            grids[r].write_local("v", grids[r].local_cells().astype(np.float64))
        check_structure(grids, o)
    for g in grids:
        g.close()


def test_cell_data_moves_with_refinement():
    """Surviving cells keep their data, new cells start at zero, refined
    parents and removed children stay readable until
    clear_refined_unrefined_data (dccrg.hpp:3519-3543, 5550-5567); halos run
    on the rebuilt plans."""
    length, M, per = (4, 4, 2), 2, (True, True, False)
    o = AmrOracle(length, M, per, 1, 2)
    grids = make_ranks(length, M, per, 1, 2)
    for g in grids:
        g.add_field("v", np.float64)
        loc = g.local_cells()
        g.write_local("v", loc.astype(np.float64) * 0.5)
    for c in (6, 11, 27):
        r = o.owner(c)
        assert grids[r].refine_completely(c) == o.refine_completely(r, c)
    new = stop_all(grids)
    want = o.stop_refining()
    for r, g in enumerate(grids):
        assert [int(c) for c in new[r]] == want[r]
        loc = g.local_cells()
        vals = g.read_local("v")
        isnew = np.isin(loc, new[r])
        assert np.all(vals[isnew] == 0)
        assert np.array_equal(vals[~isnew], loc[~isnew].astype(np.float64) * 0.5)
        # refined parents stay readable on their own rank
        for c in (6, 11, 27):
            if o.owner(c) == r and int(c) not in o.leaves:
                assert g.read_cells("v", [c])[0][0] == c * 0.5
        # children inherit the parent's value, as tests/advection/adapter.hpp:240-262 does
        par = np.array([g.mapping.get_parent(int(c)) for c in new[r]], dtype=np.uint64)
        if par.size:
            g.write_cells("v", new[r], np.concatenate(g.read_cells("v", par)))
        g.clear_refined_unrefined_data()
        if par.size:
            with pytest.raises(D.DccrgxError):
                g.read_cells("v", par[:1])
    # halo over the rebuilt plans: ghost values = the owners' values
    buf = {}
    for r, g in enumerate(grids):
        for p, ids in g.get_cells_to_send().items():
            buf[(r, p)] = dict(zip(ids, np.concatenate(g.read_cells("v", ids))))
    for r, g in enumerate(grids):
        for p, ids in g.get_cells_to_receive().items():
            assert p != r
            for c in ids:
                assert c in buf[(p, r)]
    # unrefine everything back where possible
    for r, g in enumerate(grids):
        for c in g.local_cells():
            if o.level(int(c)) == 1:
                assert g.unrefine_completely(int(c)) == o.unrefine_completely(r, int(c))
    stop_all(grids)
    o.stop_refining()
    for r, g in enumerate(grids):
        rem = g.get_removed_cells()
        assert [int(c) for c in rem] == o.get_removed_cells(r)
        if rem.size:
            # removed children still readable; their parents are new (zero) cells
            assert np.all(np.concatenate(g.read_cells("v", rem)) != 0)
            par = np.unique([g.mapping.get_parent(int(c)) for c in rem]).astype(np.uint64)
            assert np.all(np.concatenate(g.read_cells("v", par)) == 0)
    check_structure(grids, o)
    for g in grids:
        g.close()


def test_uniform_grid_switches_layout_on_refine():
    """A grid initialised without a leaf list (uniform layout) keeps its
    level-0 data when the first refine request converts it."""
    length, M, per = (6, 5, 4), 1, (False, True, True)
    o = AmrOracle(length, M, per, 1, 1)
    (g,) = make_ranks(length, M, per, 1, 1)
    g.add_field("a", np.uint32)
    ids = g.local_cells()
    g.write_local("a", (ids % 7).astype(np.uint32))
    assert g.info.uniform == 1
    assert g.refine_completely(33) == o.refine_completely(0, 33)
    assert g.info.uniform == 1  # the switch waits for the collective stop_refining
    new = g.stop_refining()
    assert g.info.uniform == 0
    assert [int(c) for c in new] == o.stop_refining()[0]
    loc = g.local_cells()
    vals = g.read_local("a")
    keep = ~np.isin(loc, new)
    assert np.array_equal(vals[keep], (loc[keep] % 7).astype(np.uint32))
    check_structure([g], o)
    g.close()


@pytest.mark.parametrize("cells,M,steps", [(16, 2, 5), (12, 1, 4)])
def test_adaptive_advection_matches_oracle(cells, M, steps):
    """tests/advection/2d.cpp with adaptation every step (adapt_n = 1):
    pre-refinement, then solve / check_for_adaptation / apply / adapt_grid.
    Leaf sets equal the oracle's after every step; densities within 1e-12
    relative (fp64, the north star's bound); time steps equal."""
    from dccrg_amd import advection as A
    from oracle.dccrg_amr import AdvectionAmrOracle
    rel, thr, sens, cfl = 0.025, 0.25, 0.5, 0.5
    ref = AdvectionAmrOracle(cells, M, 1, rel, thr, sens, cfl)
    ctx = D.Context(0, 0, 1)
    g = (D.Dccrg().set_initial_length((cells, cells, 1)).set_maximum_refinement_level(M)
         .set_periodic(True, True, False).set_neighborhood_length(0).initialize(ctx))
    g.add_advection_fields()
    geom = A.geometry_2d(g)
    A.initialize(g, geom)
    for _ in range(M):
        sets = A.check_for_adaptation(g, rel / M, thr, sens)
        A.adapt_grid(g, geom, *sets)
        A.initialize(g, geom)

    def compare(tag):
        rc, ra = ref.arrays()
        assert [int(c) for c in g.local_cells()] == rc, tag
        rho = g.read_local("density")
        assert np.max(np.abs(rho - ra[0])) <= 1e-12 * np.max(np.abs(ra[0])), tag

    compare("prerefined")
    dt = g.max_time_step()
    assert abs(dt - ref.dt) <= 1e-15 * ref.dt
    for s in range(steps):
        g.update_copies_of_remote_neighbors(fields=["density"])
        sets = A.check_for_adaptation(g, rel / M, thr, sens)
        # the three sets themselves (device sibling-group pass) equal the
        # reference loop's, cell for cell
        want = ref.check_for_adaptation()[0]
        for got, w in zip(sets, want):
            assert [int(c) for c in got] == list(w), f"step {s}"
        g.advect_step(cfl * dt)
        A.adapt_grid(g, geom, *sets)
        dt = g.max_time_step()
        ref.step()
        compare(f"step {s}")
        assert abs(dt - ref.dt) <= 1e-15 * ref.dt
    g.close()
    ctx.close()


def test_layout_switch_is_collective():
    """A request for a remote or non-existent cell switches nothing; ranks
    switch together inside stop_refining, also when only one rank asked."""
    length, M, per = (6, 5, 4), 1, (False, True, True)
    o = AmrOracle(length, M, per, 1, 2)
    grids = make_ranks(length, M, per, 1, 2)
    remote = int(grids[1].local_cells()[0])
    assert not grids[0].refine_completely(remote)
    assert not grids[0].refine_completely(10 ** 9)
    assert all(g.info.uniform == 1 for g in grids)
    new = stop_all(grids)
    assert all(g.info.uniform == 1 for g in grids) and all(n.size == 0 for n in new)
    assert grids[1].refine_completely(remote) == o.refine_completely(1, remote)
    assert grids[0].info.uniform == 1
    new = stop_all(grids)
    want = o.stop_refining()
    assert all(g.info.uniform == 0 for g in grids)
    for r in range(2):
        assert [int(c) for c in new[r]] == want[r]
    check_structure(grids, o)
    for g in grids:
        g.close()


def test_explicit_storage_is_per_rank():
    """Fields of a refined grid hold the rank's local cells, its ghosts and
    retired cells only -- not the whole grid (the reference stores data
    only for local cells and copies of remote neighbors)."""
    length, M, per = (8, 8, 8), 1, (True, True, True)
    P = 4
    grids = make_ranks(length, M, per, 1, P)
    for g in grids:
        g.add_field("a", np.float64)
    r0 = int(grids[0].local_cells()[3])
    grids[0].refine_completely(r0)
    stop_all(grids)
    total = sum(g.n_local for g in grids)
    for g in grids:
        nghost = len(g.remote_cells())
        retired = 1 if g is grids[0] else 0
        assert g.info.n_slots == g.n_local + nghost + retired
        assert g.info.n_slots < total
    # a user neighborhood lies inside the default one (dccrg.hpp:6573-6618),
    # so its ghosts already have slots; data stays put
    for g in grids:
        vals = g.local_cells().astype(np.float64)
        g.write_local("a", vals)
        items = [(1, 1, 1), (-1, -1, -1), (0, 0, 1)]
        assert g.add_neighborhood(7, items)
        assert np.array_equal(g.read_local("a"), vals)
        ghosts = set(int(c) for c in g.remote_cells()) | set(int(c) for c in g.remote_cells(7))
        g._refresh_info()
        assert g.info.n_slots == g.n_local + len(ghosts) + (1 if g is grids[0] else 0)
    for g in grids:
        g.close()


@pytest.mark.parametrize("P", [2, 3])
def test_adaptive_advection_multirank(P):
    """tests/advection/2d.cpp with adapt_n = 1 on P ranks (driven in one
    process; ghosts move through the same pack / unpack plans the RCCL path
    uses).  Per-rank leaf sets and densities match the oracle's P-rank run
    (check_for_adaptation depends on which neighbors are local)."""
    from dccrg_amd import advection as A
    from oracle.dccrg_amr import AdvectionAmrOracle
    from test_gpu_explicit import loopback
    cells, M, steps = 16, 2, 4
    rel, thr, sens, cfl = 0.025, 0.25, 0.5, 0.5
    ref = AdvectionAmrOracle(cells, M, P, rel, thr, sens, cfl)
    grids = []
    for r in range(P):
        c = D.Context(0, r, P)
        g = (D.Dccrg().set_initial_length((cells, cells, 1)).set_maximum_refinement_level(M)
             .set_periodic(True, True, False).set_neighborhood_length(0).initialize(c))
        g._keep = c
        g.add_advection_fields()
        grids.append(g)
    geoms = [A.geometry_2d(g) for g in grids]

    def init_all():
        for g, geom in zip(grids, geoms):
            A.initialize(g, geom, update=False)
        loopback(grids, list(A.ALL))

    def adapt_all(sets):
        for g, s in zip(grids, sets):
            A.request_adaptation(g, *s)
        reqs = [g.amr_requests() for g in grids]
        union = [np.unique(np.concatenate([q[k] for q in reqs])).astype(np.uint64) for k in range(4)]
        A.finish_adaptation_all(grids, geoms, union)
        loopback(grids, list(A.ALL))

    init_all()
    for _ in range(M):
        adapt_all([A.check_for_adaptation(g, rel / M, thr, sens) for g in grids])
        init_all()

    def compare(tag):
        rc, ra = ref.arrays()
        pos = {c: i for i, c in enumerate(rc)}
        assert sorted(int(c) for g in grids for c in g.local_cells()) == rc, tag
        scale = np.max(np.abs(ra[0]))
        for r, g in enumerate(grids):
            loc = [int(c) for c in g.local_cells()]
            assert loc == [c for c in rc if ref.o.owner(c) == r], tag
            rho = g.read_local("density")
            want = ra[0][[pos[c] for c in loc]]
            assert np.max(np.abs(rho - want), initial=0.0) <= 1e-12 * scale, tag

    compare("prerefined")
    dt = min(g.max_time_step() for g in grids)
    assert abs(dt - ref.dt) <= 1e-15 * ref.dt
    for s in range(steps):
        loopback(grids, ["density"])
        sets = [A.check_for_adaptation(g, rel / M, thr, sens) for g in grids]
        for g in grids:
            g.calculate_fluxes(cfl * dt, True)
            g.calculate_fluxes(cfl * dt, False)
            g.apply_fluxes()
        adapt_all(sets)
        dt = min(g.max_time_step() for g in grids)
        ref.step()
        compare(f"step {s}")
        assert abs(dt - ref.dt) <= 1e-15 * ref.dt
    for g in grids:
        g.close()


@pytest.mark.gpu
def test_calls_between_prepare_and_finish_are_refused():
    """while a two-phase stop_refining is prepared (the new fields
    and neighborhoods are built aside, the data already moved), field creation,
    field writes, new neighborhoods, halos, stencils and solvers return
    DCCRGX_ESTATE; finishing then commits the oracle's grid."""
    import torch

    import dccrg_amd as D
    from dccrg_amd import _capi as X
    from oracle.dccrg_amr import AmrOracle
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    length, M, per, hood = (4, 3, 2), 1, (True, False, True), 1
    o = AmrOracle(length, M, per, hood, 1)
    ctx = D.Context(0, 0, 1)
    g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
         .set_neighborhood_length(hood).initialize(ctx))
    try:
        for f in ("a", "b", "n"):
            g.add_field(f, np.uint32)
        g.write_local("a", np.ones(g.n_local, dtype=np.uint32))
        for c in (3, 7, 20):
            assert g.refine_completely(c) == o.refine_completely(0, c)
        st, err = g.stop_refining_prepare()
        assert st == X.DCCRGX_OK, err
        with pytest.raises(D.DccrgxError) as e:
            g.add_field("late", np.uint32)
        assert e.value.code == X.DCCRGX_ESTATE
        for call in (lambda: g.write_local("a", np.zeros(g.n_local, dtype=np.uint32)),
                     lambda: g.add_neighborhood(7, [[1, 0, 0], [-1, 0, 0]]),
                     lambda: g.start_remote_neighbor_copy_updates(fields=["a"]),
                     lambda: g.gol_step("a", "b", "n")):
            with pytest.raises(D.DccrgxError) as e:
                call()
            assert e.value.code == X.DCCRGX_ESTATE
        # every other entry point that writes field data, request
        # flags or retired data is refused too (the C-ABI directly)
        L, h = D.lib(), g._h
        fid = np.array([g.field_id("a")], dtype=np.int32)
        fp = fid.ctypes.data_as(X._i32p)
        res = np.zeros(4, dtype=np.int32)
        rp = res.ctypes.data_as(X._i32p)
        ids = np.array([5, 6], dtype=np.uint64)
        buf = np.zeros(4096, dtype=np.uint8)
        nbytes = np.zeros(1, dtype=np.uintp)
        refused = {
            "halo_self": lambda: L.dccrgx_halo_self(h, 0, fp, 1),
            "halo_pack_to": lambda: L.dccrgx_halo_pack_to(h, 0, fp, 1, 0, buf.ctypes.data, buf.size,
                                                          nbytes.ctypes.data_as(X._szp)),
            "halo_unpack_from": lambda: L.dccrgx_halo_unpack_from(h, 0, fp, 1, 0, buf.ctypes.data, 0),
            "exchange_start": lambda: L.dccrgx_exchange_start(h, 0, None, None, None, None),
            "refine_completely": lambda: L.dccrgx_refine_completely(h, 5, rp),
            "unrefine_completely": lambda: L.dccrgx_unrefine_completely(h, 5, rp),
            "dont_unrefine": lambda: L.dccrgx_dont_unrefine(h, 5, rp),
            "dont_refine": lambda: L.dccrgx_dont_refine(h, 5, rp),
            "amr_request_cells": lambda: L.dccrgx_amr_request_cells(h, 0, ids.ctypes.data_as(X._u64p), 2, rp),
            "amr_copy_from_parents": lambda: L.dccrgx_amr_copy_from_parents(h, fp, 1),
            "amr_average_children": lambda: L.dccrgx_amr_average_children(h, fp, 1),
            "clear_refined_unrefined_data": lambda: L.dccrgx_clear_refined_unrefined_data(h),
        }
        for name, call in refused.items():
            assert call() == X.DCCRGX_ESTATE, name
        g.stop_refining_finish(True)
        want = o.stop_refining()
        assert [int(c) for c in g.get_new_cells()] == want[0]
        assert [int(c) for c in g.local_cells()] == o.cells()
        g.add_field("late", np.uint32)  # allowed again
        g.gol_step("a", "b", "n")
    finally:
        g.close()
        ctx.close()


def test_ids_of_64_bits():
    """A 1x1x1 grid at the largest refinement level it allows (21): its ids
    need all 64 bits, so the device decisions sort their id lists without
    the list tags (amr_dev.hip amr_dev_decide); refines and an unrefine
    against the oracle."""
    o = AmrOracle((1, 1, 1), -1, hood_length=1, comm_size=1)
    assert o.M == 21
    grids = make_ranks((1, 1, 1), -1, (False, False, False), 1, 1)
    g = grids[0]
    for rnd in range(4):
        cells = o.cells()
        if rnd < 3:
            c = max(cells)  # the deepest cell
            assert g.refine_completely(c) == o.refine_completely(0, c)
        else:
            c = cells[-1]
            assert g.unrefine_completely(c) == o.unrefine_completely(0, c)
        got = stop_all(grids)
        want = o.stop_refining()
        assert [int(x) for x in got[0]] == want[0]
        assert [int(x) for x in g.get_removed_cells()] == o.get_removed_cells(0)
        g.clear_refined_unrefined_data()
        check_structure(grids, o)
    g.close()
