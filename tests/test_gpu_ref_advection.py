"""GPU: the device advection program against the REFERENCE's own solver
source.  oracle/_ref/ref_advection is tests/advection/{solve,adapter,
initialize,cell}.hpp compiled where they lie over this repository's drop-in
dccrg.hpp (oracle/ref_advection_main.cpp drives them as tests/advection/2d.cpp
does); it runs here on the GPU box, then the device path (dccrg_amd.advection
+ the advect/AMR kernels) runs the same program.  Leaf sets must be equal after
every step, densities within 1e-12 of the largest, time steps within 1e-12
relative (the device gathers each cell's face fluxes in a different order
than the reference's scatter; SURVEY 8(d) parity gate).  The last case is
configs[2] itself: 400 x 400, maximum level 2, adapting every step."""
import os
import subprocess

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from dccrg_amd import advection as A  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "ref_advection")
MPI_LIB = "/opt/conda/lib"


def reference_run(n, M, steps, adapt_n, out):
    env = dict(os.environ)
    env["LD_LIBRARY_PATH"] = "/usr/lib/x86_64-linux-gnu:" + MPI_LIB
    r = subprocess.run([BIN, str(n), str(M), str(steps), str(adapt_n), out], env=env, timeout=600,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(out, "rb").read()
    states, at = [], 0
    while at < len(raw):
        step, = np.frombuffer(raw, dtype=np.uint64, count=1, offset=at)
        dt, = np.frombuffer(raw, dtype=np.float64, count=1, offset=at + 8)
        k, = np.frombuffer(raw, dtype=np.uint64, count=1, offset=at + 16)
        rec = np.frombuffer(raw, dtype=np.uint8, count=16 * int(k), offset=at + 24).reshape(-1, 16)
        ids = rec[:, :8].copy().view(np.uint64).ravel()
        rho = rec[:, 8:].copy().view(np.float64).ravel()
        states.append((int(step), float(dt), ids, rho))
        at += 24 + 16 * int(k)
    return states


def device_run(n, M, steps, adapt_n, fused=False):
    """fused: the adaptation sets stay on the device (A.check_and_request,
    then finish_adaptation after the solve), as bench.py's adaptive loop."""
    rel, thr, sens, cfl = 0.025, 0.25, 0.5, 0.5
    ctx = D.Context(0, 0, 1)
    g = (D.Dccrg().set_initial_length((n, n, 1)).set_maximum_refinement_level(M)
         .set_periodic(True, True, False).set_neighborhood_length(0).initialize(ctx))
    g.add_advection_fields()
    geom = A.geometry_2d(g)
    A.initialize(g, geom)
    for _ in range(M):
        A.adapt_grid(g, geom, *A.check_for_adaptation(g, rel / M, thr, sens))
        A.initialize(g, geom)
    dt = g.max_time_step()
    states = [(0, dt, g.local_cells().copy(), g.read_local("density").copy())]
    for step in range(steps):
        g.update_copies_of_remote_neighbors(fields=["density"])
        adapt = adapt_n > 0 and step % adapt_n == 0
        sets = None
        if adapt and fused:
            A.check_and_request(g, rel / M, thr, sens)
        elif adapt:
            sets = A.check_for_adaptation(g, rel / M, thr, sens)
        g.advect_step(cfl * dt)
        if adapt and fused:
            A.finish_adaptation(g, geom)
        elif adapt:
            A.adapt_grid(g, geom, *sets)
        if adapt:
            dt = g.max_time_step()
        states.append((step + 1, dt, g.local_cells().copy(), g.read_local("density").copy()))
    g.close()
    ctx.close()
    return states


@pytest.mark.skipif(not os.path.exists(BIN), reason="oracle/_ref/ref_advection is built where /root/reference is")
@pytest.mark.parametrize("n,M,steps,adapt_n", [(20, 2, 12, 1), (40, 2, 8, 1), (32, 1, 10, 2), (24, 0, 10, 0),
                                              (64, 2, 24, 1), (400, 2, 8, 1)])
def test_device_matches_reference_solver(tmp_path, n, M, steps, adapt_n):
    ref = reference_run(n, M, steps, adapt_n, str(tmp_path / "ref.bin"))
    dev = device_run(n, M, steps, adapt_n)
    assert len(ref) == len(dev) == steps + 1
    for (s0, dt0, ids0, rho0), (s1, dt1, ids1, rho1) in zip(ref, dev):
        assert s0 == s1
        assert np.array_equal(ids0, ids1), f"leaf sets differ after step {s0}"
        scale = max(np.abs(rho0).max(), 1e-300)
        assert np.abs(rho0 - rho1).max() <= 1e-12 * scale, f"density after step {s0}"
        assert abs(dt0 - dt1) <= 1e-12 * abs(dt0), f"dt after step {s0}"


@pytest.mark.skipif(not os.path.exists(BIN), reason="oracle/_ref/ref_advection is built where /root/reference is")
@pytest.mark.parametrize("n,M,steps,adapt_n", [(20, 2, 12, 1), (64, 2, 24, 1), (400, 2, 8, 1)])
def test_incremental_rebuild_matches_reference_solver(tmp_path, lib_options, n, M, steps, adapt_n):
    """The same runs with the incremental rebuild forced (the library picks it
    above 2^20 leaves): neighbors_of rows and, on one rank, the stencil rows
    the face lists come from are copied for untouched leaves and remapped
    (explicit.hip nof_incremental, k_st_inc_fill)."""
    lib_options("incremental", 1)
    ref = reference_run(n, M, steps, adapt_n, str(tmp_path / "ref.bin"))
    dev = device_run(n, M, steps, adapt_n)
    assert len(ref) == len(dev) == steps + 1
    for (s0, dt0, ids0, rho0), (s1, dt1, ids1, rho1) in zip(ref, dev):
        assert np.array_equal(ids0, ids1), f"leaf sets differ after step {s0}"
        scale = max(np.abs(rho0).max(), 1e-300)
        assert np.abs(rho0 - rho1).max() <= 1e-12 * scale, f"density after step {s0}"


@pytest.mark.skipif(not os.path.exists(BIN), reason="oracle/_ref/ref_advection is built where /root/reference is")
@pytest.mark.parametrize("n,M,steps,adapt_n", [(20, 2, 12, 1), (64, 2, 24, 1), (400, 2, 8, 1)])
def test_device_resident_requests_match_reference_solver(tmp_path, n, M, steps, adapt_n):
    """The adaptive loop as bench.py runs it: check_for_adaptation and the
    request loops with the sets on the device (dccrgx_advect_adapt_requests),
    the data rules in one call (dccrgx_amr_adapter_data_rules)."""
    ref = reference_run(n, M, steps, adapt_n, str(tmp_path / "ref.bin"))
    dev = device_run(n, M, steps, adapt_n, fused=True)
    assert len(ref) == len(dev) == steps + 1
    for (s0, dt0, ids0, rho0), (s1, dt1, ids1, rho1) in zip(ref, dev):
        assert np.array_equal(ids0, ids1), f"leaf sets differ after step {s0}"
        scale = max(np.abs(rho0).max(), 1e-300)
        assert np.abs(rho0 - rho1).max() <= 1e-12 * scale, f"density after step {s0}"
        assert abs(dt0 - dt1) <= 1e-12 * abs(dt0), f"dt after step {s0}"


@pytest.mark.parametrize("n,M,steps", [(40, 2, 10), (128, 2, 6)])
def test_device_resident_requests_equal_host_sets(n, M, steps):
    """Bit for bit: the device-resident sets give the same leaves and
    densities as the sets through host memory (no reference binary needed)."""
    a = device_run(n, M, steps, 1, fused=False)
    b = device_run(n, M, steps, 1, fused=True)
    for (s0, dt0, ids0, rho0), (s1, dt1, ids1, rho1) in zip(a, b):
        assert np.array_equal(ids0, ids1), s0
        assert np.array_equal(rho0.view(np.uint64), rho1.view(np.uint64)), s0
        assert dt0 == dt1
