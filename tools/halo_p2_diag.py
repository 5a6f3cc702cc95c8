"""Diagnostic: basic_cell_data halo KAT (7x13x11 periodic, hood 2) with 2
ranks driven in one process (pack_to / unpack_from loopback): mismatching
received ghosts per rank."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_gpu_parity import loopback_halo, make_grid  # noqa: E402

for P in (2, 3):
    grids = [make_grid((7, 13, 11), (True, True, True), 2, 0, r, P) for r in range(P)]
    for g in grids:
        g.add_field("id", np.uint64)
        g.write_local("id", g.local_cells())
    loopback_halo(grids, ["id"])
    for r, g in enumerate(grids):
        recv = sorted(set(c for v in g.get_cells_to_receive().values() for c in v))
        got = np.concatenate(g.read_cells("id", recv))
        bad = [(c, int(v)) for c, v in zip(recv, got) if int(v) != c]
        print(P, r, "recv", len(recv), "remote", len(g.remote_cells()), "bad", len(bad), bad[:10], flush=True)
