"""bench.py's advection_large line with the explicit kernels visiting the
cells in id order and in Morton order (test option adv_order), same grid
(GPU): python tools/adv_order_cmp.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import bench  # noqa: E402
import dccrg_amd as D  # noqa: E402
from dccrg_amd.grid import set_test_option  # noqa: E402

ctx = D.Context(0, 0, 1)
for order in [int(x) for x in os.environ.get("ADV_ORDERS", "0,1,0,1").split(",")]:
    set_test_option("adv_order", order)
    r = bench.advection_large(ctx, D)
    print(json.dumps({"adv_order": order, "us_per_step": r["us_per_step"], "frac": r["frac"]}), flush=True)
ctx.close()
