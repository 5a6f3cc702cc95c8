"""Narrow down a failure seen only on the system HIP runtime: a grid built
after an adaptive advection grid was closed.  usage: rt_bisect.py MODE
  init   advection grid initialised, closed, then the 792-leaf grid
  adapt  advection grid pre-refined (adapt twice), closed, then the 792-leaf grid
  keep   as adapt, advection grid kept open"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import dccrg_amd as D  # noqa: E402
from dccrg_amd import advection as A  # noqa: E402

mode = sys.argv[1]
ctx = D.Context(0, 0, 1)
rel, thr, sens, M = 0.025, 0.25, 0.5, 2
g = (D.Dccrg().set_initial_length((400, 400, 1)).set_maximum_refinement_level(M)
     .set_periodic(True, True, False).set_neighborhood_length(0).initialize(ctx))
g.add_advection_fields()
geom = A.geometry_2d(g)
A.initialize(g, geom)
if mode in ("adapt", "keep"):
    for _ in range(M):
        A.adapt_grid(g, geom, *A.check_for_adaptation(g, rel / M, thr, sens))
        A.initialize(g, geom)
print(mode, "advection leaves", g.n_local, flush=True)
if mode != "keep":
    g.close()
pl, _, _ = bench.poisson3d_leaves()
for attempt in range(3):
    try:
        h = (D.Dccrg().set_initial_length((8, 8, 8)).set_maximum_refinement_level(2)
             .set_periodic(True, True, True).set_neighborhood_length(0).initialize(ctx, leaves=pl))
        print(mode, "attempt", attempt, "ok", h.n_local, flush=True)
        h.close()
    except Exception as e:  # noqa: BLE001
        print(mode, "attempt", attempt, "FAILED", e, flush=True)
