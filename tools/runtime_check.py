"""Which HIP runtime the process runs on, and configs[4]'s Poisson solve on it.

torch ships its own libamdhip64.so with the same soname as /opt/rocm's, so
the library that is loaded first (import order) serves the whole process.
usage: python tools/runtime_check.py [torch-first]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1 and sys.argv[1] == "torch-first":
    import torch  # noqa: F401
import numpy as np  # noqa: E402

import bench  # noqa: E402
import dccrg_amd as D  # noqa: E402

D.lib()
maps = open("/proc/self/maps").read()
print("runtime:", sorted({l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}), flush=True)
ctx = D.Context(0, 0, 1)
pl, pidx, plv = bench.poisson3d_leaves()
L0 = np.array([2 * np.pi / 8, np.pi / 8, 8 * np.pi / 8])
g = (D.Dccrg().set_initial_length((8, 8, 8)).set_maximum_refinement_level(2)
     .set_periodic(True, True, True).set_neighborhood_length(0).initialize(ctx, leaves=pl))
print("leaves", g.n_local, len(pl), flush=True)
for f in ("rhs", "solution", "length_x", "length_y", "length_z"):
    g.add_field(f, np.float64)
pln = L0[None, :] / (2.0 ** plv)[:, None]
pc = pidx * (L0 / 4)[None, :] + pln / 2
g.write_local("rhs", -(81.0 / 16.0) * np.sin(pc[:, 0]) * np.cos(2 * pc[:, 1]) * np.sin(pc[:, 2] / 4))
for k, a in enumerate(("length_x", "length_y", "length_z")):
    g.write_local(a, pln[:, k])
lc = g.local_cells()
print("local cells equal leaves:", np.array_equal(lc, pl), flush=True)
s = D.PoissonSolve(g)
g.write_local("solution", np.zeros(len(pl)))
print("solve", s.solve(pl), flush=True)
