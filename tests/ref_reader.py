"""Helpers: run the reference's own grid-data-file reader
(tests/restart/dc2vtk.cpp, built where it lies by `make -C oracle ref` into
oracle/_ref/restart_dc2vtk) and parse the VTK it writes."""
import os
import shutil
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "restart_dc2vtk")


def available() -> bool:
    return os.path.exists(BIN) and os.path.exists("/opt/conda/lib/libmpi.so")


def read_with_reference(path: str):
    """(corner points (n, 8, 3) as printed, is_alive per cell) in file order."""
    assert path.endswith(".dc")
    env = dict(os.environ)
    env["LD_LIBRARY_PATH"] = "/usr/lib/x86_64-linux-gnu:/opt/conda/lib"
    r = subprocess.run([BIN, path], capture_output=True, text=True, env=env, timeout=300,
                       cwd=os.path.dirname(path) or ".")
    assert r.returncode == 0, r.stdout + r.stderr
    vtk = path[:-2] + "vtk"
    assert os.path.exists(vtk), "the reference reader rejected the file: " + r.stdout + r.stderr
    lines = open(vtk).read().split("\n")
    i = next(k for k, l in enumerate(lines) if l.startswith("POINTS"))
    npts = int(lines[i].split()[1])
    pts = np.array([[float(v) for v in lines[i + 1 + k].split()] for k in range(npts)]).reshape(-1, 8, 3)
    j = next(k for k, l in enumerate(lines) if l.startswith("LOOKUP_TABLE"))
    alive = np.array([int(lines[j + 1 + k]) for k in range(npts // 8)], dtype=np.int64)
    return pts, alive


def expected_corners(cells, length, max_ref_lvl, start, l0):
    """Cell corners from the mapping (min corner index, level) in the order
    dc2vtk prints them (x fastest over min/max)."""
    from oracle import dccrg_oracle as O
    m = O.Mapping(length, max_ref_lvl)
    idx, lvl = m.ids_to_indices(np.asarray(cells, dtype=np.uint64))
    l0 = np.asarray(l0, dtype=np.float64)
    ln = l0[None, :] / (2.0 ** lvl.astype(np.float64))[:, None]
    mn = np.asarray(start)[None, :] + idx.astype(np.float64) * (l0 / float(2 ** m.max_ref_lvl))[None, :]
    mx = mn + ln
    out = np.zeros((len(cells), 8, 3))
    for k, (ax, ay, az) in enumerate([(0, 0, 0), (1, 0, 0), (0, 1, 0), (1, 1, 0), (0, 0, 1), (1, 0, 1), (0, 1, 1),
                                      (1, 1, 1)]):
        out[:, k, 0] = np.where(ax, mx[:, 0], mn[:, 0])
        out[:, k, 1] = np.where(ay, mx[:, 1], mn[:, 1])
        out[:, k, 2] = np.where(az, mx[:, 2], mn[:, 2])
    return out


def cleanup(path):
    for p in (path, path[:-2] + "vtk"):
        if os.path.exists(p):
            os.remove(p)
    shutil.rmtree(path + ".d", ignore_errors=True)
