"""Interleaved A/B of the batched get_indices kernel builds (DCCRGX_MAP_VARIANT
= ids per lane per pass; 1 = k_ids_to_indices_v) on 2^26 random ids of a
2048^3 grid at max level 10, HIP-event timed; 36 algorithmic bytes per id."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccrg_amd as D  # noqa: E402

m = D.Mapping((2048, 2048, 2048), 10)
nid = 1 << 26
gen = torch.Generator(device="cuda").manual_seed(1)
ids = torch.randint(1, 1 << 62, (nid,), device="cuda", dtype=torch.int64, generator=gen)
for r in range(3):
    for v in ("1", "2", "4", "8"):
        os.environ["DCCRGX_MAP_VARIANT"] = v
        m.ids_to_indices(ids)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            m.ids_to_indices(ids)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"round {r} variant {v}: {ms:.3f} ms, {36 * nid / (ms * 1e-3) / 1e9:.0f} GB/s", flush=True)
