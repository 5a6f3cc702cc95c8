"""bench.py's advection_large line alone (GPU)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import bench  # noqa: E402
import dccrg_amd as D  # noqa: E402

ctx = D.Context(0, 0, 1)
print(json.dumps(bench.advection_large(ctx, D), indent=1), flush=True)
ctx.close()
