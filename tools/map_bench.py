"""bench.py's mapping line alone: Mapping::get_indices + get_refinement_level
(dccrgx_map_ids_to_indices) on 2^26 random ids of a 2048^3 grid at max level
10, event-timed over 10 calls, 3 repeats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dccrg_amd import _capi  # noqa: E402

if os.environ.get("MAP_LIB"):  # A/B runs against another build of the library
    _capi.LIB_PATH = os.environ["MAP_LIB"]
import dccrg_amd as D  # noqa: E402

dev = torch.device("cuda", 0)
m = D.Mapping((2048, 2048, 2048), 10)
nid = 1 << 26
gen = torch.Generator(device=dev).manual_seed(1)
ids = torch.randint(1, 1 << 62, (nid,), device=dev, dtype=torch.int64, generator=gen)
m.ids_to_indices(ids)
torch.cuda.synchronize(dev)
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        m.ids_to_indices(ids)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / 10
    print(f"{os.path.basename(_capi.LIB_PATH)} {ms:.4f} ms per call, {36 * nid / (ms * 1e-3) / 1e9:.0f} GB/s, frac {36 * nid / (ms * 1e-3) / 8e12:.3f}",
          flush=True)
