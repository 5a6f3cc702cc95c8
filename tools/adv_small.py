"""configs[2]'s solver steps (bench.py's `advection` line) alone: wall time
per step and the host time spent in the advect_step call, to tell a host-bound
loop from a device-bound one (run under rocprofv3 --kernel-trace --stats for
the kernel's own duration)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from dccrg_amd import _capi  # noqa: E402

if os.environ.get("MAP_LIB"):  # A/B runs against another build of the library
    _capi.LIB_PATH = os.environ["MAP_LIB"]
import dccrg_amd as D  # noqa: E402
from dccrg_amd import advection as A  # noqa: E402

ctx = D.Context(0, 0, 1)
rel, thr, sens, cfl, M = 0.025, 0.25, 0.5, 0.5, 2
N = int(os.environ.get("ADV_N", "400"))


def run():
    g = (D.Dccrg().set_initial_length((N, N, 1)).set_maximum_refinement_level(M)
         .set_periodic(True, True, False).set_neighborhood_length(0).initialize(ctx))
    g.add_advection_fields()
    geom = A.geometry_2d(g)
    A.initialize(g, geom)
    for _ in range(M):
        A.adapt_grid(g, geom, *A.check_for_adaptation(g, rel / M, thr, sens))
        A.initialize(g, geom)
    dt_adv = g.max_time_step()
    for _ in range(20):
        g.advect_step(cfl * dt_adv)
    ctx.synchronize()
    for rep in range(3):
        steps, host = 200, 0.0
        t0 = time.perf_counter()
        for _ in range(steps):
            a = time.perf_counter()
            g.advect_step(cfl * dt_adv)
            host += time.perf_counter() - a
        ctx.synchronize()
        dt = time.perf_counter() - t0
        print(f"leaves {g.n_local} wall {dt / steps * 1e6:.2f} us/step, "
              f"host in advect_step {host / steps * 1e6:.2f} us", flush=True)
    rho = g.read_local("density").copy()
    g.close()
    return rho


run()
ctx.close()
