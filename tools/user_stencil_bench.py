"""bench.py's user_stencil_gol line alone (GPU): python tools/user_stencil_bench.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if os.environ.get("US_LIB"):  # A/B runs against another build of the example library
    bench.US_LIB = os.environ["US_LIB"]
import dccrg_amd as D  # noqa: E402

ctx = D.Context(0, 0, 1)
print(json.dumps(bench.user_stencil_gol(ctx, D)), flush=True)
ctx.close()
