"""configs[2]'s adaptive loop alone (for rocprofv3 and phase timing): the
pre-refined 400x400x1 grid of tests/advection/2d.cpp, then ADAPT_STEPS steps
of bench.py's loop (b): ghost update, check_for_adaptation, solve, adapt_grid,
max_time_step.  Prints ms per step."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if not os.environ.get("ADAPT_NO_TORCH"):
    # as bench.py and the tests: torch first, so its bundled HIP runtime
    # serves the process (ADAPT_NO_TORCH=1: /opt/rocm's, the library's own)
    import torch  # noqa: F401
import dccrg_amd as D  # noqa: E402
from dccrg_amd import advection as A  # noqa: E402
from dccrg_amd import _capi as X  # noqa: E402
from dccrg_amd._capi import check, lib  # noqa: E402
import numpy as np  # noqa: E402

if os.environ.get("ADAPT_INCREMENTAL"):  # force the incremental (1) or the full (0) list rebuild
    from dccrg_amd.grid import set_test_option
    set_test_option("incremental", int(os.environ["ADAPT_INCREMENTAL"]))
ctx = D.Context(0, 0, 1)
rel, thr, sens, cfl, M = 0.025, 0.25, 0.5, 0.5, 2
rel = float(os.environ.get("ADAPT_REL", rel))  # larger grids: smaller differences between neighbors
NX = int(os.environ.get("ADAPT_N", "400"))  # cells per side (configs[2]: 400)
g = (D.Dccrg().set_initial_length((NX, NX, 1)).set_maximum_refinement_level(M)
     .set_periodic(True, True, False).set_neighborhood_length(0).initialize(ctx))
g.add_advection_fields()
geom = A.geometry_2d(g)
A.initialize(g, geom)
for _ in range(M):
    A.adapt_grid(g, geom, *A.check_for_adaptation(g, rel / M, thr, sens))
    A.initialize(g, geom)
dt = g.max_time_step()
g.update_copies_of_remote_neighbors(fields=list(A.ALL))
steps = int(os.environ.get("ADAPT_STEPS", "20"))
per = []
seg = os.environ.get("ADAPT_SEG")  # per-phase times, synchronised after each phase (diagnosis; 2: adapt split)
segs = []
for _ in range(steps):
    t0 = time.perf_counter()
    ts = [t0]

    def mark():
        if seg:
            ctx.synchronize()
            ts.append(time.perf_counter())
    g.update_copies_of_remote_neighbors(fields=["density"])
    mark()
    if os.environ.get("ADAPT_HOST_SETS"):  # the sets through host memory (check_for_adaptation)
        sets = A.check_for_adaptation(g, rel / M, thr, sens)
    else:
        sets = None
        A.check_and_request(g, rel / M, thr, sens)
    mark()
    g.advect_step(cfl * dt)
    mark()
    if seg == "2":  # adapt_grid in its parts
        if sets is not None:
            A.request_adaptation(g, *sets)
        mark()
        g.stop_refining()
        mark()
        g.get_removed_cells()
        fd = np.array([g.field_id("density")], dtype=np.int32)
        mark()
        check(lib().dccrgx_amr_copy_from_parents(g._h, fd.ctypes.data_as(X._i32p), fd.size))
        mark()
        check(lib().dccrgx_amr_average_children(g._h, fd.ctypes.data_as(X._i32p), fd.size))
        mark()
        g.clear_refined_unrefined_data()
        mark()
        A._velocities_lengths(g, geom)
        mark()
        g.update_copies_of_remote_neighbors(fields=list(A.ALL))
        mark()
    elif sets is not None:
        A.adapt_grid(g, geom, *sets)
        mark()
    else:
        A.finish_adaptation(g, geom)
        mark()
    dt = g.max_time_step()
    mark()
    per.append((time.perf_counter() - t0) * 1e3)
    if seg:
        segs.append([(b - a) * 1e3 for a, b in zip(ts, ts[1:])])
ctx.synchronize()
if seg:
    n = max(len(segs) - 4, 1)
    names = ("ghost", "check", "advect") + (("request", "stop_refining", "removed list", "from parents",
                                                                 "average", "clear", "geometry", "update")
                                            if seg == "2" else ("adapt",)) + ("dt",)
    print(f"phases ({', '.join(names)}) ms: " + " ".join(
        f"{sum(x[i] for x in segs[4:]) / n:.3f}" for i in range(len(names))), flush=True)
print("ms/step " + " ".join(f"{x:.2f}" for x in per), flush=True)
print(f"leaves {g.n_local} mean of last {max(steps - 4, 1)}: "
      f"{sum(per[4:]) / max(len(per[4:]), 1):.2f} ms", flush=True)
g.close()
ctx.close()
