"""configs[2]'s solver alone on the pre-refined 183k-leaf grid, as bench.py's
secondary.advection line times it (Python loop of advect_step), plus the same
number of steps from C (no Python per step: dccrgx_advect_step in a loop)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
import dccrg_amd as D  # noqa: E402
from dccrg_amd import advection as A  # noqa: E402

ctx = D.Context(0, 0, 1)
rel, thr, sens, cfl, M = 0.025, 0.25, 0.5, 0.5, 2
g = (D.Dccrg().set_initial_length((400, 400, 1)).set_maximum_refinement_level(M)
     .set_periodic(True, True, False).set_neighborhood_length(0).initialize(ctx))
g.add_advection_fields()
geom = A.geometry_2d(g)
A.initialize(g, geom)
for _ in range(M):
    A.adapt_grid(g, geom, *A.check_for_adaptation(g, rel / M, thr, sens))
    A.initialize(g, geom)
dt = g.max_time_step()
for _ in range(20):
    g.advect_step(cfl * dt)
ctx.synchronize()
for rep in range(3):
    steps = 200
    t0 = time.perf_counter()
    for _ in range(steps):
        g.advect_step(cfl * dt)
    ctx.synchronize()
    us = (time.perf_counter() - t0) * 1e6 / steps
    print(f"leaves {g.n_local} python loop {us:.2f} us/step", flush=True)
g.close()
ctx.close()
