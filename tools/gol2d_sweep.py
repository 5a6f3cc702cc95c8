"""Interleaved A/B of the 2-D (LB == 1) stencil builds on configs[1]
(16384 x 16384, periodic x y) in ONE process: DCCRGX_GOL2D_VARIANT x
DCCRGX_GOL_WGS, several rounds, median kernel GB/s (12 B per cell)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccrg_amd as D  # noqa: E402

n = int(os.environ.get("SWEEP_N", "16384"))
variants = os.environ.get("SWEEP_VARIANTS", "0,4,8,16").split(",")
wgs = os.environ.get("SWEEP_WGS", "2048,4096,8192").split(",")
rounds = int(os.environ.get("SWEEP_ROUNDS", "3"))
K = int(os.environ.get("SWEEP_STEPS", "20"))

ctx = D.Context(0, 0, 1)
g = (D.Dccrg().set_initial_length((n, n, 1)).set_neighborhood_length(1).set_maximum_refinement_level(0)
     .set_periodic(True, True, False).initialize(ctx))
for f in ("a", "b", "c"):
    g.add_field(f, np.uint32)
D.lib().dccrgx_field_init_hash(g._h, g.field_id("a"), 200)
res = {}
for r in range(rounds):
    for v in variants:
        for w in wgs:
            os.environ["DCCRGX_GOL2D_VARIANT"] = v
            os.environ["DCCRGX_GOL_WGS"] = w
            g.gol_step("a", "b", "c")
            ctx.synchronize()
            g.kernel_timer(reset=1)
            t0 = time.perf_counter()
            cur, nxt = "a", "b"
            for _ in range(K):
                g.gol_step(cur, nxt, "c")
                cur, nxt = nxt, cur
            ctx.synchronize()
            wall = time.perf_counter() - t0
            ms, launches = g.kernel_timer(reset=0)
            gbs = 12 * g.n_local * K / (ms * 1e-3) / 1e9
            res.setdefault(f"{v}/wgs{w}", []).append((gbs, wall / K * 1e3))
            print(f"round {r} G={v} wgs={w}: kernel {gbs:.0f} GB/s, step {wall / K * 1e3:.3f} ms", flush=True)
summary = {k: {"median_GBs": float(np.median([x[0] for x in v])), "max_GBs": float(max(x[0] for x in v)),
               "median_step_ms": float(np.median([x[1] for x in v]))} for k, v in res.items()}
print(json.dumps(summary, indent=1))
