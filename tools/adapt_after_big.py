"""Adaptive advection loop timing (as bench.py's advection_adaptive), with
and without a large grid allocated and freed first (pool state check)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import dccrg_amd as D  # noqa: E402
from dccrg_amd import advection as A  # noqa: E402

ctx = D.Context(0, 0, 1)
if len(sys.argv) > 1 and sys.argv[1] == "big":
    n = 2048
    big = (D.Dccrg().set_initial_length((n, n, n)).set_neighborhood_length(1)
           .set_maximum_refinement_level(0).set_periodic(False, False, True).initialize(ctx))
    for f in ("alive_a", "alive_b", "count"):
        big.add_field(f, np.uint32)
    big.gol_step("alive_a", "alive_b", "count")
    ctx.synchronize()
    big.close()
rel, thr, sens, cfl, M = 0.025, 0.25, 0.5, 0.5, 2
g = (D.Dccrg().set_initial_length((400, 400, 1)).set_maximum_refinement_level(M)
     .set_periodic(True, True, False).set_neighborhood_length(0).initialize(ctx))
g.add_advection_fields()
geom = A.geometry_2d(g)
A.initialize(g, geom)
for _ in range(M):
    A.adapt_grid(g, geom, *A.check_for_adaptation(g, rel / M, thr, sens))
    A.initialize(g, geom)
dt_adv = g.max_time_step()
for _ in range(51):
    g.advect_step(cfl * dt_adv)
ctx.synchronize()
g.update_copies_of_remote_neighbors(fields=list(A.ALL))
per = []
t0 = time.perf_counter()
for _ in range(20):
    ts = time.perf_counter()
    g.update_copies_of_remote_neighbors(fields=["density"])
    sets = A.check_for_adaptation(g, rel / M, thr, sens)
    t1 = time.perf_counter()
    g.advect_step(cfl * dt_adv)
    ctx.synchronize()
    t2 = time.perf_counter()
    A.request_adaptation(g, *sets)
    t3 = time.perf_counter()
    from dccrg_amd import _capi as X
    new = g.stop_refining()
    rem = g.get_removed_cells()
    ctx.synchronize()
    tq = [time.perf_counter()]
    fd = np.array([g.field_id("density")], dtype=np.int32)
    X.check(D.lib().dccrgx_amr_copy_from_parents(g._h, fd.ctypes.data_as(X._i32p), fd.size))
    tq.append(time.perf_counter())
    X.check(D.lib().dccrgx_amr_average_children(g._h, fd.ctypes.data_as(X._i32p), fd.size))
    tq.append(time.perf_counter())
    g.clear_refined_unrefined_data()
    A._velocities_lengths(g, geom)
    ctx.synchronize()
    tq.append(time.perf_counter())
    g.update_copies_of_remote_neighbors(fields=list(A.ALL))
    ctx.synchronize()
    tq.append(time.perf_counter())
    nn, nr = new.size, rem.size
    t4 = time.perf_counter()
    if os.environ.get("DCCRGX_TIMING"):
        print(f"finish: stop_refining+lists {1e3*(tq[0]-t3):.1f} copy_from_parents {1e3*(tq[1]-tq[0]):.1f} "
              f"average {1e3*(tq[2]-tq[1]):.1f} clear+geometry {1e3*(tq[3]-tq[2]):.1f} "
              f"update {1e3*(tq[4]-tq[3]):.1f}", file=sys.stderr, flush=True)
    dt_adv = g.max_time_step()
    per.append((time.perf_counter() - ts) * 1e3)
    if os.environ.get("DCCRGX_TIMING"):
        print(f"step check {1e3*(t1-ts):.1f} advect {1e3*(t2-t1):.1f} requests {1e3*(t3-t2):.1f} "
              f"finish {1e3*(t4-t3):.1f} maxdt {1e3*(time.perf_counter()-t4):.1f} new {nn} removed {nr}",
              file=sys.stderr, flush=True)
ctx.synchronize()
print(sys.argv[1:] or ["plain"], "ms/step", round((time.perf_counter() - t0) * 1e3 / 20, 2),
      " ".join(f"{x:.1f}" for x in per), flush=True)
g.close()
ctx.close()
