"""GPU: the neighbor gather for user stencils (dccrgx_gather_neighbors) --
with every cell's data equal to its id (examples/basic_cell_data.cpp's KAT
idea), the gathered values must be exactly the get_neighbors_of ids, in list
order, on uniform and refined grids, at 1-3 ranks (ghosts after the halo)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from oracle import dccrg_oracle as O  # noqa: E402

DEV = torch.device("cuda", 0)


def ranks(length, M, per, hood, P, leaves=None):
    out = []
    for r in range(P):
        c = D.Context(0, r, P)
        g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
             .set_neighborhood_length(hood).initialize(c, leaves=leaves))
        g._keep = c
        out.append(g)
    return out


def loopback(grids, fields):
    msgs = {}
    for r, g in enumerate(grids):
        for p in g.get_cells_to_send():
            buf = torch.empty(1 << 22, dtype=torch.uint8, device=DEV)
            torch.cuda.synchronize()
            msgs[(r, p)] = (buf, g.pack_to(p, buf.data_ptr(), buf.numel(), fields=fields))
            g.ctx.synchronize()
    for r, g in enumerate(grids):
        g.halo_self(fields=fields)
        for p in g.get_cells_to_receive():
            buf, nb = msgs[(p, r)]
            g.unpack_from(p, buf.data_ptr(), nb, fields=fields)
        g.ctx.synchronize()


def refined(length, n_ref, seed):
    rng = np.random.default_rng(seed)
    m = O.Mapping(length, 1)
    n0 = int(np.prod(length))
    ref = set(int(v) for v in rng.choice(np.arange(1, n0 + 1), size=n_ref, replace=False))
    leaves = []
    for c in range(1, n0 + 1):
        leaves += m.get_all_children(c) if c in ref else [c]
    return sorted(leaves)


CASES = [((10, 8, 6), (False, False, False), 1, 0, 1, None),
         ((10, 8, 6), (True, True, True), 1, 0, 3, None),
         ((12, 5, 1), (True, False, False), 2, 0, 2, None),
         ((6, 6, 6), (False, True, True), 0, 0, 3, None),
         ((1, 1, 1), (True, True, True), 1, 0, 1, None),
         ((6, 5, 4), (True, True, False), 1, 1, 1, 40),
         ((6, 5, 4), (False, True, True), 1, 1, 3, 30),
         ((8, 8, 1), (True, True, False), 0, 1, 2, 20),
         # neighborhood length 3: 342 items, beyond the LDS-record kernel (192)
         ((9, 8, 7), (True, True, True), 3, 0, 1, None),
         ((10, 9, 8), (False, True, True), 3, 0, 2, None)]


@pytest.mark.parametrize("length,per,hood,M,P,n_ref", CASES)
@pytest.mark.parametrize("kind", ["u64", "u8x72"])
def test_gathered_values_are_neighbor_ids(length, per, hood, M, P, n_ref, kind):
    leaves = refined(length, n_ref, 3) if n_ref else None
    grids = ranks(length, M, per, hood, P, leaves)
    for g in grids:
        loc = g.local_cells()
        if kind == "u64":
            g.add_field("d", np.uint64)
            g.write_local("d", loc)
        else:  # 72 opaque bytes: the id in the first 8, a pattern after
            g.add_field("d", np.dtype((np.uint8, 72)))
            v = np.zeros((loc.size, 72), dtype=np.uint8)
            v[:, :8] = loc.astype(np.uint64).view(np.uint8).reshape(-1, 8)
            v[:, 8:] = (np.arange(64, dtype=np.uint8)[None, :] + loc.astype(np.uint8)[:, None])
            g.write_local("d", v)
    loopback(grids, ["d"])
    for g in grids:
        loc = g.local_cells()
        if not loc.size:
            continue
        row, vals = g.gather_neighbors("d")
        row = row.cpu().numpy()
        vals = vals.cpu().numpy()
        nrow, nids, _ = g.neighbors_of(loc)
        assert np.array_equal(row.astype(np.uint64), nrow)
        if kind == "u64":
            assert np.array_equal(vals.view(np.uint64), nids)
        else:
            rec = vals.reshape(-1, 72)
            assert np.array_equal(rec[:, :8].copy().view(np.uint64).ravel(), nids)
            assert np.array_equal(rec[:, 8:], np.arange(64, dtype=np.uint8)[None, :] + nids.astype(np.uint8)[:, None])
    for g in grids:
        g.close()


def test_remote_query_cell_is_rejected():
    grids = ranks((6, 6, 6), 0, (False, False, False), 1, 2)
    g = grids[0]
    g.add_field("d", np.uint32)
    other = grids[1].local_cells()[:1]
    with pytest.raises(D.DccrgxError) as e:
        g.gather_neighbors("d", cells=other)
    assert e.value.code == 7
    for x in grids:
        x.close()
