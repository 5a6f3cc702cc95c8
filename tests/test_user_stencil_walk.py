"""CPU: include/dccrgx_stencil.hpp's uniform neighbor walk (the code device
functors run, compiled for the host by tests/cpp/stencil_walk.cpp) gives
every cell its neighbors_of in the reference's iteration-cache order
(dccrg.hpp:11590-11640) -- the oracle's find_neighbors_of / find_neighbors_to
lists grouped by oracle.iteration_cache_lists -- on all three paths: cells no
boundary reaches (fixed slot distances), cells near a non-periodic boundary
only, and cells near a periodic wrap (key selection; 1- and 2-cell periodic
axes give self and duplicate ids).  Rank slabs (lo, hi) check ghost slots."""
import os
import subprocess

import numpy as np
import pytest

from oracle import dccrg_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"

CASES = [  # length (z > 1: canonical axes are x, y, z), periodic, items (None: the cube of hood length h)
    ((10, 8, 6), (False, False, False), 1, None),
    ((10, 8, 6), (True, True, True), 1, None),
    ((7, 6, 5), (True, False, True), 2, None),
    ((2, 3, 2), (True, True, True), 1, None),
    ((1, 1, 3), (True, True, True), 1, None),
    ((6, 5, 4), (True, True, True), 2, [[-2, 0, 1], [1, 1, 1], [0, -1, 0], [2, -2, 2]]),
    ((6, 5, 4), (False, True, False), 1, [[-1, 0, 1], [1, 1, 1], [0, -1, 0], [1, -1, 0], [0, 0, -1]]),
]


@pytest.fixture(scope="module")
def walker(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc absent")
    out = str(tmp_path_factory.mktemp("walk") / "stencil_walk")
    subprocess.check_call([HIPCC, "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "stencil_walk.cpp"), "-o", out])
    return out


def cube(h):
    return [[x, y, z] for z in range(-h, h + 1) for y in range(-h, h + 1) for x in range(-h, h + 1)
            if (x, y, z) != (0, 0, 0)]


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("case", CASES)
def test_walk_order(walker, case, P):
    length, per, h, items = case
    items = cube(h) if items is None else items
    n = int(np.prod(length))
    S = length[0] * length[1]
    og = O.Grid(length, 0, per, h, list(range(1, n + 1)))
    it = np.array(items, dtype=np.int32)
    for r in range(P):
        lo, hi = n * r // P, n * (r + 1) // P  # rank slabs of cells (not slice-aligned)
        cbase = lo // S - 3                    # storage slice 0 three slices below the first local one
        inp = f"{length[0]} {length[1]} {length[2]} {int(per[0])} {int(per[1])} {int(per[2])} {lo} {hi} {cbase} " \
              f"{len(items)} " + " ".join(f"{a} {b} {c}" for a, b, c in items)
        res = subprocess.run([walker], input=inp, capture_output=True, text=True, timeout=120)
        assert res.returncode == 0, res.stderr
        lines = res.stdout.split("\n")
        assert len([x for x in lines if x]) == hi - lo
        for line in lines:
            if not line:
                continue
            v = [int(t) for t in line.split()]
            cell, k = v[0], v[1]
            got = [(v[2 + 4 * e], (v[3 + 4 * e], v[4 + 4 * e], v[5 + 4 * e])) for e in range(k)]
            want = O.iteration_cache_lists(og.find_neighbors_of(cell, it), og.find_neighbors_to(cell, -it))[0]
            assert got == want, (cell, got, want)
