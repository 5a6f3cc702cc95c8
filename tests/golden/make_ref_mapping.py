#!/usr/bin/env python3
"""Generate tests/golden/ref_mapping.npz from the REFERENCE's own Mapping and
Cartesian_Geometry classes (dccrg_mapping.hpp, dccrg_cartesian_geometry.hpp),
built from /root/reference by `make -C oracle ref` (oracle/ref_mapping_main.cpp).

Run in the container that holds /root/reference; the committed .npz is data
(inputs and the reference's outputs), read by tests/test_ref_mapping.py on any
machine.  Grids are the SURVEY 8(c)(1) list plus the Poisson and advection
geometries: ids at every level boundary, error ids and seeded random ids per
level; get_cell_from_indices on seeded in-range and out-of-range queries.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
BIN = os.path.join(REPO, "oracle", "_ref", "ref_mapping")
OUT = os.path.join(HERE, "ref_mapping.npz")

# (name, length, max_ref_lvl (-1 = maximum possible), start, level-0 cell length)
CASES = [
    ("c1_10x10x1_l0", (10, 10, 1), 0, (0.0, 0.0, 0.0), (1.0, 1.0, 1.0)),
    ("t_3x3x1_l1", (3, 3, 1), 1, (0.0, 0.0, 0.0), (1.0, 1.0, 1.0)),
    ("c3_400x400x1_l2", (400, 400, 1), 2, (0.0, 0.0, 0.0), (1.0 / 400, 1.0 / 400, 1.0 / 400)),
    ("t_100x200x300_l13", (100, 200, 300), 13, (-1.5, 2.25, 1e3), (0.1, 0.3, 7.0)),
    ("c4_2048c_l0", (2048, 2048, 2048), 0, (0.0, 0.0, 0.0), (1.0, 1.0, 1.0)),
    ("c4_2048c_l10", (2048, 2048, 2048), 10, (0.0, 0.0, 0.0), (1.0 / 2048, 1.0 / 2048, 1.0 / 2048)),
    ("c5_8c_l2", (8, 8, 8), 2, (0.0, 0.0, 0.0), (2 * np.pi / 8, np.pi / 8, 8 * np.pi / 8)),
    ("t_1x1x1_lmax", (1, 1, 1), -1, (0.0, 0.0, 0.0), (1.0, 1.0, 1.0)),
    ("t_5x7x3_lmax", (5, 7, 3), -1, (3.0, -4.0, 0.5), (0.25, 0.5, 2.0)),
    ("t_16384x16384x1_l0", (16384, 16384, 1), 0, (0.0, 0.0, 0.0), (1.0, 1.0, 1.0)),
]
N_RANDOM_PER_LEVEL = 12
N_QUERIES = 160


def level_first_ids(length, M):
    n0 = length[0] * length[1] * length[2]
    first, c = [], 1
    for lvl in range(M + 2):
        first.append(c)
        c += n0 * (8 ** lvl)
    return first  # first[M + 1] = last_cell + 1


def case_inputs(length, M, seed):
    rng = np.random.default_rng(seed)
    first = level_first_ids(length, M)
    last = first[M + 1] - 1
    ids = [0, 1, 2, last, last + 1, last + 2, (1 << 32) - 1, 1 << 32, (1 << 63), (1 << 64) - 1]
    for lvl in range(M + 1):
        lo, hi = first[lvl], first[lvl + 1] - 1
        ids += [lo, lo + 1, hi - 1, hi]
        ids += [int(v) for v in rng.integers(lo, hi + 1, size=N_RANDOM_PER_LEVEL, dtype=np.uint64)]
    ids = np.array([v % (1 << 64) for v in ids], dtype=np.uint64)
    # get_cell_from_indices queries: in range, on the upper edge, beyond it; levels -1..M+1
    top = np.array(length, dtype=np.uint64) * np.uint64(1 << M)
    q = np.zeros((N_QUERIES, 4), dtype=np.uint64)
    for i in range(N_QUERIES):
        kind = i % 4
        for k in range(3):
            if kind == 3 and k == i % 3:
                q[i, k] = top[k] + np.uint64(rng.integers(0, 3))
            elif kind == 2:
                q[i, k] = top[k] - np.uint64(1)
            else:
                q[i, k] = np.uint64(rng.integers(0, int(top[k])))
        q[i, 3] = np.uint64(int(rng.integers(-1, M + 2)) % (1 << 64))
    return ids, q


def run_case(length, M, start, l0, ids, q):
    args = [BIN] + [str(v) for v in length] + [str(M)] + [repr(float(v)) for v in start] + \
        [repr(float(v)) for v in l0]
    payload = (np.array([ids.size], dtype=np.uint64).tobytes() + ids.tobytes() +
               np.array([q.shape[0]], dtype=np.uint64).tobytes() + q.tobytes())
    out = subprocess.run(args, input=payload, stdout=subprocess.PIPE, check=True).stdout
    hdr = np.frombuffer(out[:24], dtype=np.int64)
    rec_bytes = 28 * 8 + 12 * 8
    body = out[24:24 + rec_bytes * ids.size]
    raw = np.frombuffer(body, dtype=np.uint8).reshape(ids.size, rec_bytes)
    rec = raw[:, :224].copy().view(np.uint64).reshape(ids.size, 28)[:, :25]
    geo = raw[:, 224:].copy().view(np.float64).reshape(ids.size, 12)
    qcell = np.frombuffer(out[24 + rec_bytes * ids.size:], dtype=np.uint64)
    assert qcell.size == q.shape[0]
    return hdr, rec, geo, qcell


def main():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    arrays, meta = {}, []
    for ci, (name, length, M, start, l0) in enumerate(CASES):
        Mq = M
        if M < 0:  # the program resolves -1 to the maximum possible level
            hdr, _, _, _ = run_case(length, M, start, l0, np.zeros(0, dtype=np.uint64),
                                    np.zeros((0, 4), dtype=np.uint64))
            Mq = int(hdr[0])
        ids, q = case_inputs(length, Mq, 1000 + ci)
        hdr, rec, geo, qcell = run_case(length, M, start, l0, ids, q)
        meta.append({"name": name, "length": list(length), "max_ref_lvl_arg": M, "max_ref_lvl": int(hdr[0]),
                     "last_cell": int(np.uint64(hdr[1])), "max_possible": int(hdr[2]),
                     "start": list(start), "level_0_cell_length": [float(v) for v in l0]})
        arrays[f"{name}.ids"] = ids
        arrays[f"{name}.rec"] = rec
        arrays[f"{name}.geo"] = geo
        arrays[f"{name}.q"] = q
        arrays[f"{name}.qcell"] = qcell
    arrays["meta"] = np.array(json.dumps({
        "source": "reference dccrg_mapping.hpp / dccrg_cartesian_geometry.hpp built by oracle/Makefile ref",
        "rec_columns": ["ix", "iy", "iz", "level(i64)", "length_in_indices", "parent", "level_0_parent",
                        "child", "children[8]", "siblings[8]", "get_cell_from_indices(get_indices)"],
        "geo_columns": ["length[3]", "center[3]", "min[3]", "max[3]"],
        "q_columns": ["ix", "iy", "iz", "level(i64)"],
        "cases": meta}))
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT}: {len(CASES)} cases, {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    sys.exit(main())
