#!/usr/bin/env python3
"""Headline benchmark: cell updates/s including the halo exchange, weak-scaled.

Workload (BASELINE.json configs[3]): 3-D game of life on a
uniform 2048 x 2048 x (2048 * N) level-0 grid, neighborhood length 1 (26
neighbors), periodic in z (a ring of z-slabs, the reference block
partition), random initial state (splitmix64(id) % 1000 < 200).  One step =
remote-neighbor halo start, inner cells, halo wait, outer cells (the overlap
pattern of tests/game_of_life/scalability3d.cpp:122-166), on every rank.

Run: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, halo over RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "cell updates/sec incl. halo exchange (1/2/4/8 GPU) + % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
BYTES_PER_CELL = 12    # read is_alive 4 + write is_alive 4 + write live_neighbor_count 4


def cpu_baseline(seconds: float = 10.0):
    """The oracle's port of the reference hot loop (explicit neighbor lists,
    examples/game_of_life.cpp:54-79), one host core, on a bounded sample."""
    from oracle import dccrg_oracle as O
    L = (96, 96, 96)
    n = L[0] * L[1] * L[2]
    lists = O.GolLists(L, (False, False, True), 1)
    alive = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 200)
    count = np.zeros(n, dtype=np.uint32)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        lists.step(alive, count)
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": steps * n / dt, "unit": "cell-updates/s", "cores": 1, "kind": "port",
            "sample": f"{L[0]}x{L[1]}x{L[2]} uniform grid, hood 1, periodic z, {steps} steps "
                      f"({dt:.1f} s) of oracle/dccrg_oracle.c dox_gol_count+apply over "
                      f"face-graph-walk neighbor lists"}


def pmc_traffic(kernel: str, cells_per_launch: int):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of the
    same kernel and launch size (tools/summarize_prof.py; FETCH_SIZE and
    WRITE_SIZE in separate passes, gfx950 corrections applied), or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json")), key=os.path.getmtime):
        try:
            s = json.load(open(f))
        except (OSError, ValueError):
            continue
        if kernel in s.get("kernel", "") and s.get("cells_per_launch") == cells_per_launch:
            best = (s["traffic_bytes_per_launch"], os.path.relpath(f, ROOT))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=2048, help="cells per axis per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist
    import dccrg_amd as D

    ndev = torch.cuda.device_count()
    device = local_rank % max(ndev, 1)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = D.Context(device, rank, world)
    if world > 1:
        uid = [D.Context.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(uid[0])

    n = args.n
    length = (n, n, n * world)
    t_init = time.perf_counter()
    grid = (D.Dccrg().set_initial_length(length).set_neighborhood_length(1)
            .set_maximum_refinement_level(0).set_periodic(False, False, True).initialize(ctx))
    for f in ("alive_a", "alive_b", "count"):
        grid.add_field(f, np.uint32)
    D.lib().dccrgx_field_init_hash(grid._h, grid.field_id("alive_a"), 200)
    t_init = time.perf_counter() - t_init
    n_local = grid.n_local

    def barrier():
        ctx.synchronize()
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()

    cur, nxt = "alive_a", "alive_b"
    for _ in range(args.warmup):
        grid.gol_step(cur, nxt, "count")
        cur, nxt = nxt, cur
    barrier()
    grid.kernel_timer(reset=1)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        grid.gol_step(cur, nxt, "count")
        cur, nxt = nxt, cur
    barrier()
    dt = time.perf_counter() - t0
    kern_ms, launches = grid.kernel_timer(reset=0)
    grid.kernel_timer(reset=-1)

    if world > 1:
        t = torch.tensor([dt, kern_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, kern_ms = float(t[0]), float(t[1])

    total_cells = n_local * world
    value = total_cells * args.steps / dt
    # dominant kernel: the LDS-tiled 26-neighbor stencil; algorithmic bytes =
    # 12 B per cell it updates; average launch duration from HIP events on the
    # compute stream around each launch in the timed region
    launch_bytes = BYTES_PER_CELL * n_local * args.steps
    achieved = launch_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "cell-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: alive = splitmix64(cell id) % 1000 < 200",
        "config": {
            "workload": "tests/game_of_life/scalability3d 3-D game of life, uniform "
                        f"{length[0]}x{length[1]}x{length[2]} grid, neighborhood length 1 (26 "
                        "neighbors), periodic z, block (z-slab) partition, halo over RCCL",
            "cells_per_gpu": n_local,
            "grid": list(length),
            "parallelism": f"z-slab x{world}",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": None,
            "kernel": "dccrgx::k_gol26v<8, 4, true>",
            "kernel_ms_per_step": kern_ms / args.steps,
            "launches_per_step": launches / max(args.steps, 1),
            "bytes_per_cell": BYTES_PER_CELL,
        },
        "init_s": t_init,
    }
    if launches == args.steps:  # one stencil launch per step (no remote halo split)
        t = pmc_traffic("k_gol26v<8, 4, true>", n_local)
        if t:
            line["roofline"]["traffic"] = t[0]
            line["roofline"]["traffic_source"] = t[1]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(line), flush=True)
    grid.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
