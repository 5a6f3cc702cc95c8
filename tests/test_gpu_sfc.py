"""GPU: the space-filling-curve placement (sfc.hip, dccrg.hpp:8147-8220) --
the device owner table against the oracle's, and every per-rank structure,
the halo, the game of life and refinement on SFC-placed grids against the
oracle with the same owner table."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from dccrg_amd import _capi as X  # noqa: E402
from oracle import dccrg_oracle as O  # noqa: E402
from oracle.dccrg_amr import AmrOracle  # noqa: E402

DEV = torch.device("cuda", 0)


def sfc_ranks(length, M, per, hood, P, leaves=None):
    grids = []
    for r in range(P):
        c = D.Context(0, r, P)
        g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
             .set_neighborhood_length(hood).set_initial_partition("sfc").initialize(c, leaves=leaves))
        g._keep = c
        grids.append(g)
    return grids


@pytest.mark.parametrize("L,P", [((5, 7, 3), 4), ((64, 32, 16), 8), ((3, 1, 1), 5), ((100, 100, 1), 3)])
def test_device_owner_table(L, P):
    ctx = D.Context(0, 0, 1)
    n = int(np.prod(L))
    out = np.zeros(n, dtype=np.int32)
    ln = np.array(L, dtype=np.uint64)
    X.check(D.lib().dccrgx_sfc_owners(ctx._h, ln.ctypes.data_as(X._u64p), P, out.ctypes.data_as(X._i32p)))
    assert np.array_equal(out, O.sfc_owner_table(L, P))
    ctx.close()


def check_ranks(grids, og, P):
    for r, g in enumerate(grids):
        ref = og.rank_view(r, P)
        assert g.local_cells().tolist() == ref["local"]
        assert g.inner_cells().tolist() == ref["inner"]
        assert g.outer_cells().tolist() == ref["outer"]
        assert g.remote_cells().tolist() == ref["remote"]
        assert g.get_cells_to_send() == ref["send"]
        assert g.get_cells_to_receive() == ref["recv"]


CASES = [((6, 5, 4), (True, True, True), 1, 3), ((9, 9, 1), (False, False, False), 1, 4),
         ((8, 8, 8), (True, False, True), 2, 5), ((7, 3, 5), (False, True, False), 0, 2)]


@pytest.mark.parametrize("length,per,hood,P", CASES)
def test_rank_structures_and_gol(length, per, hood, P):
    og = O.Grid(length, 0, per, hood)
    og.l0_owner = O.sfc_owner_table(length, P)
    grids = sfc_ranks(length, 0, per, hood, P)
    check_ranks(grids, og, P)
    # the game of life on the SFC placement equals the single-process run
    n = int(np.prod(length))
    a0 = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 300)
    steps = 5
    ref_a, ref_n = O.gol_reference_run(length, per, hood, a0, steps)
    for g in grids:
        for f in ("a", "b", "n"):
            g.add_field(f, np.uint32)
        g.write_local("a", a0[g.local_cells().astype(np.int64) - 1])
    cur, nxt = "a", "b"
    for _ in range(steps):
        msgs = {}
        for r, g in enumerate(grids):
            for p in g.get_cells_to_send():
                buf = torch.empty(1 << 20, dtype=torch.uint8, device=DEV)
                torch.cuda.synchronize()
                msgs[(r, p)] = (buf, g.pack_to(p, buf.data_ptr(), buf.numel(), fields=[cur]))
                g.ctx.synchronize()
        for r, g in enumerate(grids):
            g.halo_self(fields=[cur])
            for p in g.get_cells_to_receive():
                buf, nb = msgs[(p, r)]
                g.unpack_from(p, buf.data_ptr(), nb, fields=[cur])
            g.gol_compute(cur, nxt, "n")
            g.ctx.synchronize()
        cur, nxt = nxt, cur
    got_a = np.zeros(n, dtype=np.uint32)
    got_n = np.zeros(n, dtype=np.uint32)
    for g in grids:
        loc = g.local_cells().astype(np.int64) - 1
        got_a[loc] = g.read_local(cur)
        got_n[loc] = g.read_local("n")
        g.close()
    assert np.array_equal(got_a, ref_a) and np.array_equal(got_n, ref_n)


@pytest.mark.parametrize("length,M,per,hood,P,seed", [((4, 4, 2), 2, (True, True, False), 1, 3, 1),
                                                      ((5, 3, 3), 1, (False, False, True), 1, 2, 2)])
def test_refinement_keeps_sfc_owners(length, M, per, hood, P, seed):
    """Children stay with their level-0 ancestor's process (dccrg.hpp:10243-
    10693 without load balancing) under the SFC placement."""
    table = O.sfc_owner_table(length, P)
    o = AmrOracle(length, M, per, hood, P, l0_owner=table)
    grids = sfc_ranks(length, M, per, hood, P)
    rng = np.random.default_rng(seed)
    for _ in range(2):
        cells = o.cells()
        for c in rng.choice(cells, min(len(cells), 6), replace=False):
            c = int(c)
            r = o.owner(c)
            assert grids[r].refine_completely(c) == o.refine_completely(r, c)
        reqs = [g.amr_requests() for g in grids]
        union = [np.unique(np.concatenate([q[k] for q in reqs])).astype(np.uint64) for k in range(4)]
        got = D.stop_refining_all(grids, union)
        want = o.stop_refining()
        for r in range(P):
            assert [int(c) for c in got[r]] == want[r]
        assert sorted(int(c) for g in grids for c in g.local_cells()) == o.cells()
        check_ranks(grids, o.grid, P)
    for g in grids:
        g.close()


def test_partition_value_checked():
    ctx = D.Context(0, 0, 1)
    g = D.Dccrg().set_initial_length((4, 4, 4))
    g._partition = 7
    with pytest.raises(D.DccrgxError):
        g.initialize(ctx)
    ctx.close()
