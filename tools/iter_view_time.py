"""Time of the first user-stencil view after a structural change on a refined
hood-2 grid of >= 1 M leaves (dccrgx_stencil_view_get regroups the stencil
rows into the iteration cache's order, stencil.hip k_iter_rows), and of the
functor walk over it (examples/user_stencil.hip us_digest) (GPU)."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

import dccrg_amd as D  # noqa: E402
from dccrg_amd import _capi as X  # noqa: E402

L = C.CDLL(os.path.join(ROOT, "examples", "libuser_stencil.so"))
L.us_digest.argtypes = [C.c_void_p] + [C.c_int32] * 6
n = int(os.environ.get("ITER_N", "100"))
ctx = D.Context(0, 0, 1)
g = (D.Dccrg().set_initial_length((n, n, n)).set_maximum_refinement_level(1).set_periodic(True, True, True)
     .set_neighborhood_length(2).initialize(ctx))
for f, t in (("id", np.uint64), ("cid", np.uint64), ("dig", np.uint64), ("cnt", np.uint32)):
    g.add_field(f, t)
rng = np.random.default_rng(3)
for rnd in range(3):
    cells = g.local_cells()
    for c in rng.choice(cells, 2000, replace=False):
        g.refine_completely(int(c))
    g.stop_refining()
    g.clear_refined_unrefined_data()
    ctx.synchronize()
    g.write_local("id", g.local_cells())
    ctx.synchronize()
    t0 = time.perf_counter()
    v = g.stencil_view(D.DEFAULT_NEIGHBORHOOD_ID)
    ctx.synchronize()
    t1 = time.perf_counter()
    f = g.field_id
    assert L.us_digest(g._h, D.DEFAULT_NEIGHBORHOOD_ID, X.REGION_ALL, f("id"), f("cid"), f("dig"), f("cnt")) == 0
    ctx.synchronize()
    t2 = time.perf_counter()
    st = g.neighbor_list_stats()
    print(f"round {rnd}: leaves {g.n_local} stencil entries ~{int(g.read_local('cnt').sum())} "
          f"first view {1e3 * (t1 - t0):.3f} ms, functor walk {1e3 * (t2 - t1):.3f} ms, rows {st['rows']}", flush=True)
g.close()
ctx.close()
