"""GPU: the AMR-aware game of life kernels (golh.hip) against the REFERENCE's
own tests/game_of_life/solve.hpp, compiled where it lies over this
repository's drop-in dccrg.hpp (oracle/ref_gol_main.cpp, built into
oracle/_ref/).  Refined grids (cells refined once, hood 1, periodic x y):
the state of every leaf must be equal after every step."""
import os
import subprocess

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from oracle import dccrg_oracle as O  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "ref_gol")
MPI_LIB = "/opt/conda/lib"


def reference_run(lx, ly, permille, seed, steps, out):
    env = dict(os.environ)
    env["LD_LIBRARY_PATH"] = "/usr/lib/x86_64-linux-gnu:" + MPI_LIB
    r = subprocess.run([BIN, str(lx), str(ly), str(permille), str(seed), str(steps), out], env=env, timeout=600,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = np.fromfile(out, dtype=np.uint64)
    states, at = [], 0
    while at < raw.size:
        step, n = int(raw[at]), int(raw[at + 1])
        rec = raw[at + 2:at + 2 + 2 * n].reshape(-1, 2)
        states.append((step, rec[:, 0].copy(), rec[:, 1].copy()))
        at += 2 + 2 * n
    return states


def device_run(lx, ly, permille, seed, steps):
    n0 = lx * ly
    ids0 = np.arange(1, n0 + 1, dtype=np.uint64)
    refined = O.splitmix64(ids0 ^ np.uint64(seed)) % np.uint64(1000) < np.uint64(permille)
    m = O.Mapping((lx, ly, 1), 1)
    leaves = []
    for c, r in zip(ids0.tolist(), refined.tolist()):
        leaves += m.get_all_children(c) if r else [c]
    leaves = np.array(sorted(leaves), dtype=np.uint64)
    ctx = D.Context(0, 0, 1)
    g = (D.Dccrg().set_initial_length((lx, ly, 1)).set_neighborhood_length(1).set_maximum_refinement_level(1)
         .set_periodic(True, True, False).initialize(ctx, leaves=leaves))
    g.add_field("data", np.dtype((np.uint64, 9)))
    loc = g.local_cells()
    par = np.array([m.get_level_0_parent(int(c)) for c in loc], dtype=np.uint64)
    d = np.zeros((loc.size, 9), dtype=np.uint64)
    d[:, 0] = (O.splitmix64(par) % np.uint64(1000) < np.uint64(300)).astype(np.uint64)
    g.write_local("data", d)
    states = [(0, loc.copy(), d[:, 0].copy())]
    for step in range(steps):
        g.update_copies_of_remote_neighbors(fields=["data"])
        g.gol_amr_step("data")
        states.append((step + 1, g.local_cells().copy(), g.read_local("data")[:, 0].copy()))
    g.close()
    ctx.close()
    return states


@pytest.mark.skipif(not os.path.exists(BIN), reason="oracle/_ref/ref_gol is built where /root/reference is")
@pytest.mark.parametrize("lx,ly,permille,seed,steps", [(12, 10, 250, 1, 10), (24, 16, 400, 7, 12), (9, 9, 0, 3, 8),
                                                       (16, 16, 1000, 5, 6)])
def test_device_matches_reference_solver(tmp_path, lx, ly, permille, seed, steps):
    ref = reference_run(lx, ly, permille, seed, steps, str(tmp_path / "ref.bin"))
    dev = device_run(lx, ly, permille, seed, steps)
    assert len(ref) == len(dev) == steps + 1
    for (s0, i0, a0), (s1, i1, a1) in zip(ref, dev):
        assert s0 == s1
        assert np.array_equal(i0, i1), f"leaves differ at step {s0}"
        assert np.array_equal(a0, a1), f"states differ after step {s0}"
