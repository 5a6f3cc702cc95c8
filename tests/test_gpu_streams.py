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
