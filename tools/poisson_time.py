"""configs[4]'s Poisson solve alone (for rocprofv3): bench.py's 792-leaf
poisson3d grid, 50 solves."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import dccrg_amd as D  # noqa: E402

ctx = D.Context(0, 0, 1)
pl, pidx, plv = bench.poisson3d_leaves()
L0 = np.array([2 * np.pi / 8, np.pi / 8, 8 * np.pi / 8])
g = (D.Dccrg().set_initial_length((8, 8, 8)).set_maximum_refinement_level(2)
     .set_periodic(True, True, True).set_neighborhood_length(0).initialize(ctx, leaves=pl))
for f in ("rhs", "solution", "length_x", "length_y", "length_z"):
    g.add_field(f, np.float64)
pln = L0[None, :] / (2.0 ** plv)[:, None]
pc = pidx * (L0 / 4)[None, :] + pln / 2
g.write_local("rhs", -(81.0 / 16.0) * np.sin(pc[:, 0]) * np.cos(2 * pc[:, 1]) * np.sin(pc[:, 2] / 4))
for k, a in enumerate(("length_x", "length_y", "length_z")):
    g.write_local(a, pln[:, k])
s = D.PoissonSolve(g)
g.write_local("solution", np.zeros(len(pl)))
s.solve(pl)
t0 = time.perf_counter()
for _ in range(50):
    g.write_local("solution", np.zeros(len(pl)))
    it, res = s.solve(pl, cache_is_up_to_date=True)
print(f"solve_ms {(time.perf_counter() - t0) * 1e3 / 50:.3f} iterations {it} residual {res:.3e}", flush=True)
s.close()
g.close()
ctx.close()
