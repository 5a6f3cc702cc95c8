"""bench.py checks its own timed run at every N.

After the timed loop the bench reseeds the same grid with random 24^3 patches
at every rank's slab seams (rank 0's is the periodic ring wrap), tile seams
and the planes past linear index 2^32, steps K = 8 times through the same
gol_step and compares each window bit for bit with `bench.gol_box`, plus an
all-rank checksum.  Here: the checker equals the oracle (the reference's
neighbor lists and B3/S23 rule, oracle/dccrg_oracle.c), the windows cover
what they must, and on the GPU the 2-rank rehearsal passes while a corrupted
ghost plane makes the bench fail with a non-zero exit code.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import bench
from oracle import dccrg_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("dims,seed", [((12, 10, 9), 1), ((20, 20, 20), 2), ((7, 30, 11), 3), ((1, 16, 16), 4)])
def test_checker_equals_oracle(dims, seed):
    rng = np.random.default_rng(seed)
    box = (rng.random(dims[::-1]) < 0.25).astype(np.uint32)  # [z, y, x]
    for k in (1, 3, 8):
        ra, rn = O.gol_reference_run(dims, (False, False, False), 1, box.ravel(), k)
        ba, bn = bench.gol_box(box, k)
        assert np.array_equal(ba.ravel(), ra), (dims, k)
        assert np.array_equal(bn.ravel(), rn), (dims, k)


@pytest.mark.parametrize("n,world", [(2048, 1), (2048, 2), (2048, 8), (256, 2), (256, 3), (128, 8), (64, 1)])
def test_windows_cover_the_seams(n, world):
    wins = bench.check_windows(n, world)
    lz = n * world
    P, PAD = bench.CHECK_P, bench.CHECK_PAD
    # every rank's lower seam (and so the ring wrap) lies inside some patch
    for r in range(world):
        z = r * n
        assert any(1 <= (z - c[2]) % lz <= P - 1 for c, _ in wins), (r, wins)
    # pairwise disjoint windows, z modulo lz
    for i, (_, a) in enumerate(wins):
        for _, b in wins[:i]:
            assert any(a[ax][1] <= b[ax][0] or b[ax][1] <= a[ax][0] for ax in (0, 1)) or \
                all(a[2][1] <= b[2][0] + s or b[2][1] + s <= a[2][0] for s in (-lz, 0, lz))
    for c, w in wins:
        assert 0 <= c[0] <= n - P and 0 <= c[1] <= n - P
        assert w[2][1] - w[2][0] == P + 2 * PAD
    if lz * n * n > 1 << 32:  # a window holds linear index 2^32 (id 2^32 + 1)
        ids = np.concatenate([bench.window_ids(w, n, lz) for _, w in wins])
        assert (1 << 32) + 1 in set(ids.tolist())


def test_window_ids_order():
    w = [(1, 3), (0, 2), (-1, 1)]
    ids = bench.window_ids(w, 4, 8)
    # z = 7 (wrapped), 0; y = 0, 1; x = 1, 2
    want = [1 + x + 4 * (y + 4 * z) for z in (7, 0) for y in (0, 1) for x in (1, 2)]
    assert ids.tolist() == want


def _bench(gpus, extra_env=None, n=256, extra_args=()):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--n", str(n),
                        "--steps", "2", "--warmup", "1", "--no-secondary", "--no-cpu-baseline",
                        "--no-halo-payload", "--stall-timeout", "100", *extra_args],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return r, lines


@pytest.mark.gpu
@pytest.mark.parametrize("gpus,n", [(1, 256), (2, 256), (3, 256), (8, 128)])
def test_bench_self_check_passes(gpus, n):
    """8 ranks (the SCALE run's shape: 8 slab seams and the ring wrap) share
    the one GPU through the host-staged transport."""
    r, lines = _bench(gpus, n=n)
    assert r.returncode == 0, r.stderr[-3000:]
    (line,) = lines
    c = line["check"]
    assert c["bit_exact"] and c["windows_bit_exact"] and c["checksum_equal"], c
    assert c["patches"] >= 2 * gpus and c["window_cells"] > 0
    assert line["n_gpus"] == gpus


@pytest.mark.gpu
def test_bench_self_check_catches_a_bad_ghost_plane():
    r, lines = _bench(2, extra_args=["--test-corrupt-ghost"])
    assert r.returncode != 0
    (line,) = lines
    assert line["check"]["bit_exact"] is False
    assert "self-check failed" in r.stderr
