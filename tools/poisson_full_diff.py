"""Diagnostic: full Poisson solves on the device vs the oracle, per case and
iteration driver -- iteration counts, residuals and the max difference
relative to max|x| (what tests/test_gpu_poisson.py::test_poisson_full_solve
gates)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import dccrg_amd as D  # noqa: E402
import test_gpu_poisson as T  # noqa: E402

from dccrg_amd.grid import set_test_option  # noqa: E402

for path in ("solo", "solo_global", "multi", "rccl"):
    os.environ.pop("DCCRGX_TEST_RCCL", None)
    set_test_option("poisson_solo_global", 1 if path == "solo_global" else None)
    set_test_option("poisson_multi", 1 if path == "multi" else None)
    if path == "rccl":
        os.environ["DCCRGX_TEST_RCCL"] = "1"
    for name in sorted(T.CASES):
        g, sysm, cells, rhs, guess, solve, skip = T.build(name)
        s = D.PoissonSolve(g)
        g.write_local("solution", guess)
        it, res = s.solve(solve, skip)
        ref, rit, rres = sysm.solve(rhs, guess)
        got = g.read_local("solution")
        scale = max(np.abs(ref).max(), 1.0)
        print(f"{path:12s} {name:14s} it {it:4d} ref {rit:4d} res {res:.3e} ref {rres:.3e} "
              f"maxdiff/scale {np.abs(got - ref).max() / scale:.3e}", flush=True)
        s.close()
        g.close()
