"""Queries on a caller's stream stay valid across a following rebuild
(ADVICE r3, medium): the library queues the query kernels on the caller's
stream; the compute stream then waits for them (CallerStream, internal.hpp),
so the blocks a refine frees and hands out again are not reused while the
query still reads them.  A long sleep kernel queued first on the caller's
stream holds the query back until after stop_refining has run."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from dccrg_amd import _capi as X  # noqa: E402
from oracle import dccrg_oracle as O  # noqa: E402


@pytest.mark.parametrize("uniform", [False, True])
def test_query_on_caller_stream_survives_refine(uniform):
    dev = torch.device("cuda", 0)
    length, M, per, hood = (24, 24, 8), 1, (True, True, True), 1
    n0 = int(np.prod(length))
    leaves = None
    if not uniform:
        m = O.Mapping(length, M)
        cells = set(range(1, n0 + 1)) - {100}
        leaves = sorted(cells | set(m.get_all_children(100)))
    ctx = D.Context(0, 0, 1)
    g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
         .set_neighborhood_length(hood).initialize(ctx, leaves=leaves))
    try:
        q_cells = np.array(leaves if leaves else np.arange(1, n0 + 1), dtype=np.uint64)
        want_row, want_ids, want_off = g.neighbors_of(q_cells)
        cells = torch.from_numpy(q_cells.view(np.int64)).to(dev)
        q = cells.numel()
        row = torch.zeros(q + 1, dtype=torch.int64, device=dev)
        total = int(want_row[-1])
        ids = torch.zeros(total, dtype=torch.int64, device=dev)
        off = torch.zeros((total, 3), dtype=torch.int32, device=dev)
        s = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize(dev)
        with torch.cuda.stream(s):
            torch.cuda._sleep(200_000_000)  # ~0.1 s of device time ahead of the query
        X.check(D.lib().dccrgx_neighbors_of(g._h, X.DEFAULT_NEIGHBORHOOD_ID, cells.data_ptr(), q, row.data_ptr(),
                                            ids.data_ptr(), off.data_ptr(), total, s.cuda_stream))
        # a rebuild right behind it: frees the old lists and allocates new ones
        for c in (7, 300, 2000):
            g.refine_completely(c)
        g.stop_refining()
        torch.cuda.synchronize(dev)
        assert np.array_equal(row.cpu().numpy().astype(np.uint64), want_row)
        assert np.array_equal(ids.cpu().numpy().view(np.uint64), want_ids)
        assert np.array_equal(off.cpu().numpy(), want_off)
    finally:
        g.close()
        ctx.close()


@pytest.mark.parametrize("uniform", [False, True])
def test_mirror_queries_follow_torch_stream_work(uniform):
    """What's weak r5 #8: the Python mirror hands torch's current stream to
    the exports (no device-wide synchronisation around a query).  A long sleep
    and the zero fills of the result tensors are queued on torch's stream
    first -- on a side stream made current, too -- and the lists must still
    be the oracle's: the query is ordered after them on the same stream."""
    dev = torch.device("cuda", 0)
    length, M, per, hood = (12, 10, 6), 1, (True, False, True), 1
    n0 = int(np.prod(length))
    leaves = None
    if not uniform:
        m = O.Mapping(length, M)
        leaves = sorted((set(range(1, n0 + 1)) - {50}) | set(m.get_all_children(50)))
    og = O.Grid(length, M, per, hood, leaves)
    ctx = D.Context(0, 0, 1)
    g = (D.Dccrg().set_initial_length(length).set_maximum_refinement_level(M).set_periodic(*per)
         .set_neighborhood_length(hood).initialize(ctx, leaves=leaves))
    try:
        cells = np.array(leaves if leaves else np.arange(1, n0 + 1), dtype=np.uint64)
        want = [[(int(i), tuple(int(v) for v in o)) for i, o in og.find_neighbors_of(int(c))] for c in cells]
        side = torch.cuda.Stream(device=dev)
        for s in (torch.cuda.current_stream(dev), side):
            with torch.cuda.stream(s):
                torch.cuda._sleep(100_000_000)
                junk = torch.full((1 << 24,), -1, dtype=torch.int64, device=dev)  # torch work ahead of the query
                row, ids, off = g.neighbors_of(cells)
                del junk
            for i, c in enumerate(cells):
                got = [(int(ids[e]), tuple(int(v) for v in off[e])) for e in range(int(row[i]), int(row[i + 1]))]
                assert got == want[i], (int(c), got, want[i])
    finally:
        g.close()
        ctx.close()


def test_gather_on_caller_stream_follows_library_writes():
    """The entry fence of a caller-stream call (CallerStream): a field written
    by the library on its compute stream is what a gather on torch's stream
    reads, with no synchronisation in between."""
    dev = torch.device("cuda", 0)
    length = (16, 8, 4)
    n0 = int(np.prod(length))
    ctx = D.Context(0, 0, 1)
    g = (D.Dccrg().set_initial_length(length).set_periodic(True, True, True).set_neighborhood_length(1)
         .initialize(ctx))
    try:
        g.add_field("v", np.uint64)
        for rnd in range(3):
            vals = (np.arange(1, n0 + 1, dtype=np.uint64) * np.uint64(rnd + 3))
            g.write_local("v", vals)
            g.update_copies_of_remote_neighbors(fields=["v"])
            with torch.cuda.stream(torch.cuda.Stream(device=dev)):
                row, out = g.gather_neighbors("v")
                # read on the stream the result was handed over to (torch's
                # default stream is not ordered after a side stream)
                got = out.cpu().numpy().view(np.uint64)
            rr, ids, _ = g.neighbors_of(np.arange(1, n0 + 1, dtype=np.uint64))
            assert np.array_equal(got, ids * np.uint64(rnd + 3))
    finally:
        g.close()
        ctx.close()
