"""bench.secondary_host_heavy (configs[2] advection + adaptive loop, then
configs[4] Poisson) in a process without torch (system HIP runtime) or with
torch imported first (torch's bundled runtime).
usage: python tools/host_heavy_check.py [torch-first]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1 and sys.argv[1] == "torch-first":
    import torch  # noqa: F401
import bench  # noqa: E402
import dccrg_amd as D  # noqa: E402

D.lib()
print("runtime:", sorted({l.split()[-1] for l in open("/proc/self/maps").read().splitlines()
                          if "libamdhip64" in l}), flush=True)
ctx = D.Context(0, 0, 1)
r = bench.secondary_host_heavy(ctx, D)
print(json.dumps({k: {kk: v for kk, v in r[k].items() if kk != "workload"} for k in r}), flush=True)
