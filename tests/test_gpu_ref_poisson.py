"""GPU: tests/poisson/poisson1d.cpp's known-answer test on the device -- the
BiCG solver (poisson.hip) with poisson1d's own parameters (Poisson_Solve(10,
0, 1e-7, 2, 10), :167) on 1-D periodic grids along x, y and z, offset to 0 in
the last cell (:86-122), against the REFERENCE's serial 1-D solver
(tests/poisson/reference_poisson_solve.hpp built where it lies,
oracle/_ref/ref_poisson1d): 2-norms to the reference and between the three
orientations within poisson1d's threshold 3e-7 (:285-289)."""
import os
import subprocess

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "ref_poisson1d")


def reference(n):
    r = subprocess.run([BIN, str(n)], capture_output=True, timeout=120)
    assert r.returncode == 0
    return np.frombuffer(r.stdout, dtype=np.float64)


def device(n, axis, ctx):
    length = [1, 1, 1]
    length[axis] = n
    dx = 2 * np.pi / n
    g = (D.Dccrg().set_initial_length(tuple(length)).set_maximum_refinement_level(0)
         .set_periodic(True, True, True).set_neighborhood_length(0).initialize(ctx))
    for f in ("rhs", "solution", "length_x", "length_y", "length_z"):
        g.add_field(f, np.float64)
    cells = g.local_cells()
    g.write_local("rhs", np.sin((cells.astype(np.float64) - 1 + 0.5) * dx))
    g.write_local("solution", np.zeros(cells.size))
    for k, f in enumerate(("length_x", "length_y", "length_z")):
        g.write_local(f, np.full(cells.size, dx if k == axis else 1.0))
    s = D.PoissonSolve(g, 10, 0, 1e-7, 2, 10)
    s.solve(cells)
    sol = g.read_local("solution")
    s.close()
    g.close()
    return sol - sol[-1]  # offset_solution: 0 in the last cell


@pytest.mark.skipif(not os.path.exists(BIN), reason="oracle/_ref/ref_poisson1d is built where /root/reference is")
def test_poisson1d_kat():
    ctx = D.Context(0, 0, 1)
    n = 8
    while n <= 32768:
        ref = reference(n)
        sols = [device(n, axis, ctx) for axis in range(3)]
        for axis, s in enumerate(sols):
            assert np.linalg.norm(s - ref) <= 3e-7, (n, axis, np.linalg.norm(s - ref))
        for a, b in ((0, 1), (0, 2), (1, 2)):
            assert np.linalg.norm(sols[a] - sols[b]) <= 3e-7, (n, a, b)
        n *= 2
    ctx.close()
