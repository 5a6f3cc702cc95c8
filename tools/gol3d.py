"""The headline step alone (configs[3]: 3-D game of life 2048^3, hood 1,
periodic z, one GPU): kernel-timer time per step; MAP_LIB= runs another
build of the library (A/B of kernel variants on one box)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from dccrg_amd import _capi  # noqa: E402

if os.environ.get("MAP_LIB"):
    _capi.LIB_PATH = os.environ["MAP_LIB"]
import dccrg_amd as D  # noqa: E402

ctx = D.Context(0, 0, 1)
n = int(os.environ.get("GOL_N", "2048"))
g = (D.Dccrg().set_initial_length((n, n, n)).set_neighborhood_length(1)
     .set_maximum_refinement_level(0).set_periodic(False, False, True).initialize(ctx))
for f in ("a", "b", "c"):
    g.add_field(f, np.uint32)
D.lib().dccrgx_field_init_hash(g._h, g.field_id("a"), 200)
cur, nxt = "a", "b"
g.gol_step(cur, nxt, "c")
ctx.synchronize()
for rep in range(2):
    steps = 10
    g.kernel_timer(reset=1)
    t0 = time.perf_counter()
    for _ in range(steps):
        g.gol_step(cur, nxt, "c")
        cur, nxt = nxt, cur
    ctx.synchronize()
    dt = time.perf_counter() - t0
    kms, nk = g.kernel_timer(reset=0)
    g.kernel_timer(reset=-1)
    print(f"{os.path.basename(_capi.LIB_PATH)} wall {dt / steps * 1e3:.3f} ms/step, kernel timer {kms / steps:.3f} "
          f"ms/step, {12 * n ** 3 / (kms / steps * 1e-3) / 1e9:.0f} GB/s", flush=True)
g.close()
ctx.close()
