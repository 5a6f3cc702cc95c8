"""Where the adaptive advection step's time goes (configs[2], 400x400x1,
max_ref_lvl 2, adapt every step): cProfile of the host side plus the
library's phase timers (DCCRGX_TIMING=1, stderr)."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import dccrg_amd as D  # noqa: E402
from dccrg_amd import _capi as X  # noqa: E402
from dccrg_amd import advection as A  # noqa: E402

rel, thr, sens, cfl, M = 0.025, 0.25, 0.5, 0.5, 2
ctx = D.Context(0, 0, 1)
g = (D.Dccrg().set_initial_length((400, 400, 1)).set_maximum_refinement_level(M)
     .set_periodic(True, True, False).set_neighborhood_length(0).initialize(ctx))
g.add_advection_fields()
geom = A.geometry_2d(g)
A.initialize(g, geom)
for _ in range(M):
    A.adapt_grid(g, geom, *A.check_for_adaptation(g, rel / M, thr, sens))
    A.initialize(g, geom)
dt = g.max_time_step()
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3


def loop():
    global dt
    for _ in range(steps):
        g.update_copies_of_remote_neighbors(fields=["density"])
        t0 = time.perf_counter()
        sets = A.check_for_adaptation(g, rel / M, thr, sens)
        t1 = time.perf_counter()
        g.advect_step(cfl * dt)
        ctx.synchronize()
        t2 = time.perf_counter()
        tr = []
        for kind, ids in ((X.AMR_REFINE, sets[0]), (X.AMR_DONT_UNREFINE, sets[1]), (X.AMR_UNREFINE, sets[2])):
            A._request(g, kind, ids)
            tr.append(time.perf_counter())
        g._refresh_info()
        ta = time.perf_counter()
        print(f"  check {1e3*(t1-t0):.1f} requests: refine {len(sets[0])} {1e3*(tr[0]-t2):.1f} "
              f"dont_unrefine {len(sets[1])} {1e3*(tr[1]-tr[0]):.1f} unrefine {len(sets[2])} {1e3*(tr[2]-tr[1]):.1f}"
              f" refresh {1e3*(ta-tr[2]):.1f} ms", flush=True)
        new = g.stop_refining()
        g.get_removed_cells()
        ctx.synchronize()
        tb = time.perf_counter()
        fd = np.array([g.field_id("density")], dtype=np.int32)
        X.check(D.lib().dccrgx_amr_copy_from_parents(g._h, fd.ctypes.data_as(X._i32p), fd.size))
        tp = time.perf_counter()
        X.check(D.lib().dccrgx_amr_average_children(g._h, fd.ctypes.data_as(X._i32p), fd.size))
        tq = time.perf_counter()
        g.clear_refined_unrefined_data()
        ctx.synchronize()
        tc = time.perf_counter()
        print(f"  data: copy_from_parents {1e3*(tp-tb):.1f} average_children {1e3*(tq-tp):.1f} "
              f"clear {1e3*(tc-tq):.1f} ms", flush=True)
        A._velocities_lengths(g, geom)
        ctx.synchronize()
        td = time.perf_counter()
        g.update_copies_of_remote_neighbors(fields=list(A.ALL))
        t3 = time.perf_counter()
        print(f"  requests {1e3*(ta-t2):.1f} stop_refining {1e3*(tb-ta):.1f} data {1e3*(tc-tb):.1f} "
              f"velocities {1e3*(td-tc):.1f} update {1e3*(t3-td):.1f} ms (new {new.size})", flush=True)
        dt = g.max_time_step()
        print(f"cells {g.n_local} check {1e3*(t1-t0):.1f} ms solve {1e3*(t2-t1):.1f} ms adapt {1e3*(t3-t2):.1f} ms",
              flush=True)


pr = cProfile.Profile()
pr.enable()
loop()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
