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
US_LIB = os.path.join(ROOT, "examples", "libuser_stencil.so")  # tools/user_stencil_bench.py A/B runs replace it
sys.path.insert(0, ROOT)

METRIC = "cell updates/sec incl. halo exchange (1/2/4/8 GPU) + % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
BYTES_PER_CELL = 12    # read is_alive 4 + write is_alive 4 + write live_neighbor_count 4


def cpu_threads_cap():
    """Threads the CPU baseline may use: the cores this process may run on
    (its affinity mask), capped by the job's CPU share where the box states
    one (OMP_NUM_THREADS: 16 per GPU on the GPU box, whose 256 logical CPUs
    are shared by 8 GPU jobs -- the pool's rules size worker pools to that
    share, so the sweep stops there rather than at the machine's cores)."""
    h = host_cpu()
    cap = h["usable_cpus"] or 1
    share = h["omp_num_threads"]
    if share and share.isdigit() and int(share) > 0:
        cap = min(cap, int(share))
    return cap


def cpu_baseline(seconds: float = 12.0):
    """The oracle's port of the reference hot loop (explicit neighbor lists,
    examples/game_of_life.cpp:54-79) on a bounded sample, swept over OpenMP
    thread counts 1, 2, 4, ... up to cpu_threads_cap(); the best rate is the
    baseline, with its thread count, and every point is listed."""
    from oracle import dccrg_oracle as O
    L = (128, 128, 128)
    n = L[0] * L[1] * L[2]
    lists = O.GolLists(L, (False, False, True), 1)
    alive0 = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 200)
    count = np.zeros(n, dtype=np.uint32)
    cap = cpu_threads_cap()
    counts = sorted({t for t in (1, 2, 4, 8, 16, 32, 64, 128, 256) if t <= cap} | {cap})
    per = seconds / len(counts)
    sweep = {}
    best = None
    for t in counts:
        O.lib().dox_set_num_threads(t)
        alive = alive0.copy()
        lists.step(alive, count)  # warm caches and the thread pool
        steps = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < per:
            lists.step(alive, count)
            steps += 1
        dt = time.perf_counter() - t0
        rate = steps * n / dt
        sweep[str(t)] = rate
        if best is None or rate > best[0]:
            best = (rate, t, steps, dt)
    O.lib().dox_set_num_threads(cap)
    rate, threads, steps, dt = best
    return {"value": rate, "unit": "cell-updates/s", "cores": int(threads),
            "kind": "port",
            "threads_swept": sweep,
            "sample": f"{L[0]}x{L[1]}x{L[2]} uniform grid, hood 1, periodic z, {steps} steps "
                      f"({dt:.1f} s) at the best of {len(counts)} thread counts (1..{cap}) of "
                      f"oracle/dccrg_oracle.c dox_gol_count+apply over face-graph-walk neighbor lists",
            "host": host_cpu(),
            # the reference program itself cannot be built here (dccrg.hpp needs
            # Boost.TTI and Zoltan, absent from this image),
            # so its own MPI-CPU figures are the ones the survey measured (BASELINE.md
            # section 2), quoted as measured there -- not on this box
            "reference_measured": {
                "kind": "reference", "source": "BASELINE.md section 2 / SURVEY.md section 6",
                "program": "tests/game_of_life/scalability3d.cpp, unmodified, 100^3, 26 neighbors, 100 steps, "
                           "its own timer around the step loop incl. halo",
                "host": "survey container: Intel Xeon, 8 cores (1 thread/core), g++ 11.4 -O3, MPICH 3.3.2",
                "unit": "cell-updates/s", "by_ranks": {"1": 7.90e6, "2": 1.55e7, "4": 2.69e7, "8": 4.30e7}}}


def host_cpu():
    """CPU model and the cores this process may use (lscpu's model name, the
    affinity mask; on the GPU box the machine's count is larger than the
    share a one-GPU job gets)."""
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"model": model, "logical_cpus": os.cpu_count(), "usable_cpus": usable,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def profile_key(path: str):
    """Natural order of profile names by round: r3z < r3z5 < r4a (digits
    compare as numbers, a name sorts before its extensions)."""
    import re
    base = os.path.basename(path).split("_", 1)[0]
    return [int(t) if t.isdigit() else t for t in re.findall(r"\d+|\D+", base)]


def pmc_traffic(kernel: str, cells_per_launch: int):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of the
    same kernel and launch size (tools/summarize_prof.py; FETCH_SIZE and
    WRITE_SIZE in separate passes, gfx950 corrections applied), or None."""
    import glob
    best = None
    # latest round wins (natural order of the round key, not lexical)
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json")), key=profile_key):
        try:
            s = json.load(open(f))
        except (OSError, ValueError):
            continue
        if kernel in s.get("kernel", "") and s.get("cells_per_launch") == cells_per_launch:
            best = (s["traffic_bytes_per_launch"], os.path.relpath(f, ROOT))
    return best


# ---- self-check of the timed run (every N) ----------------------------------
CHECK_P = 24      # patch edge
CHECK_K = 8       # steps after seeding the patches
CHECK_PAD = CHECK_K + 1


def splitmix64(x):
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def gol_box(alive, steps):
    """The checker: 3-D game of life (26 neighbors, born on 3, survives on 2
    or 3: tests/game_of_life/scalability3d.cpp:136-165) on a [z, y, x] box
    whose outside is dead, in plain numpy.  Returns (alive, live neighbor
    count of the last step) as u32, the two fields the device step writes.
    tests/test_bench_check.py holds it to the oracle."""
    a = np.asarray(alive, dtype=np.uint8)
    cnt = np.zeros(a.shape, dtype=np.uint8)
    Z, Y, X = a.shape
    for _ in range(steps):
        p = np.pad(a, 1)
        cnt = np.zeros(a.shape, dtype=np.uint8)
        for dz in range(3):
            for dy in range(3):
                for dx in range(3):
                    if dz == dy == dx == 1:
                        continue
                    cnt += p[dz:dz + Z, dy:dy + Y, dx:dx + X]
        a = ((cnt == 3) | ((a == 1) & (cnt == 2))).astype(np.uint8)
    return a.astype(np.uint32), cnt.astype(np.uint32)


def check_windows(n: int, world: int):
    """Patch windows of the N-rank grid n x n x (n * world), periodic z:
    every rank's lower slab seam (for rank 0 the ring wrap from the last
    plane), at the x/y edges and inside, each slab's middle at a stencil tile
    seam, and -- when the grid holds more than 2^32 cells -- the planes where
    the linear index crosses 2^32.  Returns [(corner (x, y, z), window)],
    windows pairwise disjoint (z modulo n * world); a window is the patch
    padded by K + 1 cells, x and y clipped to the non-periodic box."""
    P, PAD, LZ = CHECK_P, CHECK_PAD, n * world
    cand = []
    edges = [(0, 0), (n - P, n - P), (0, n - P), (n - P, 0)]
    for r in range(world):
        z = r * n - P // 2
        cand.append((*edges[r % 4], z))
        cand.append(((n // 2 - P // 2 + 37 * r) % (n - P), (n // 3 + 53 * r) % (n - P), z))
    for r in range(world):
        xa = 256 - P // 2 if n >= 512 else n // 4
        cand.append((xa, (1024 - P // 2) % (n - P) if n > 1024 else n // 2, r * n + n // 2 - P // 2))
    if LZ * n * n > 1 << 32:
        z32 = (1 << 32) // (n * n)
        cand.append((0, 0, z32 - P // 2))
        cand.append((n - P, n - P, z32 - P // 2))

    def window(c):
        x0, y0, z0 = c
        return [(max(0, x0 - PAD), min(n, x0 + P + PAD)), (max(0, y0 - PAD), min(n, y0 + P + PAD)),
                (z0 - PAD, z0 + P + PAD)]

    def disjoint(w1, w2):
        for ax in range(3):
            (a0, a1), (b0, b1) = w1[ax], w2[ax]
            if ax < 2 and (a1 <= b0 or b1 <= a0):
                return True
            if ax == 2 and all(a1 <= b0 + s or b1 + s <= a0 for s in (-LZ, 0, LZ)):
                return True
        return False
    out = []
    for c in cand:
        w = window(c)
        if w[2][1] - w[2][0] <= LZ and all(disjoint(w, v) for _, v in out):
            out.append((c, w))
    return out


def window_ids(w, n: int, lz: int):
    """Cell ids of a window in [z, y, x] order (z modulo lz)."""
    (x0, x1), (y0, y1), (z0, z1) = w
    x = np.arange(x0, x1, dtype=np.uint64)
    y = np.arange(y0, y1, dtype=np.uint64)
    z = np.mod(np.arange(z0, z1, dtype=np.int64), lz).astype(np.uint64)
    Zg, Yg, Xg = np.meshgrid(z, y, x, indexing="ij")
    nn = np.uint64(n)
    return (Xg + nn * (Yg + nn * Zg) + np.uint64(1)).ravel()


def check_run(grid, ctx, n: int, world: int, rank: int, fields, allgather):
    """After the timed loop (outside the timing): reseed the same grid with
    empty state plus random 24^3 patches at the places of check_windows,
    step CHECK_K times through the same gol_step (halo included), and compare
    every rank's part of every window bit for bit with gol_box, plus a
    full-grid checksum (sum and splitmix64(id)-weighted sum of alive and of
    live neighbor counts, summed over ranks) against the windows' sums, so
    no cell outside the windows changed either.  `allgather(obj)` returns
    every rank's obj."""
    import dccrg_amd as D
    cur, nxt, cnt = fields
    lz = n * world
    n_local = grid.n_local
    lo = rank * n_local  # block partition: cells_per_process = n^3 exactly
    D.lib().dccrgx_field_init_hash(grid._h, grid.field_id(cur), 0)  # all dead
    rng = np.random.default_rng(1 << 20)
    wins = check_windows(n, world)
    expect = []
    for (x0, y0, z0), w in wins:
        dims = tuple(hi - lo_ for lo_, hi in w)
        box = np.zeros(dims[::-1], dtype=np.uint8)
        ox, oy, oz = x0 - w[0][0], y0 - w[1][0], z0 - w[2][0]
        box[oz:oz + CHECK_P, oy:oy + CHECK_P, ox:ox + CHECK_P] = rng.random((CHECK_P,) * 3) < 0.2
        ids = window_ids(w, n, lz)
        mine = (ids - np.uint64(1) >= np.uint64(lo)) & (ids - np.uint64(1) < np.uint64(lo + n_local))
        sel = (box.ravel() != 0) & mine
        if sel.any():
            grid.write_cells(cur, ids[sel], np.ones(int(sel.sum()), dtype=np.uint32))
        ra, rn = gol_box(box, CHECK_K)
        expect.append((ids, mine, ra.ravel(), rn.ravel()))
    for _ in range(CHECK_K):
        grid.gol_step(cur, nxt, cnt)
        cur, nxt = nxt, cur
    ctx.synchronize()
    bad = []
    sums = [0, 0, 0, 0]
    M64 = (1 << 64) - 1
    for k, (ids, mine, ra, rn) in enumerate(expect):
        with np.errstate(over="ignore"):
            mix = splitmix64(ids)
            sums[0] += int(ra.astype(np.uint64).sum())
            sums[1] = (sums[1] + int((ra.astype(np.uint64) * mix).sum(dtype=np.uint64))) & M64
            sums[2] += int(rn.astype(np.uint64).sum())
            sums[3] = (sums[3] + int((rn.astype(np.uint64) * mix).sum(dtype=np.uint64))) & M64
        if not mine.any():
            continue
        got_a = np.concatenate(grid.read_cells(cur, ids[mine]))
        got_n = np.concatenate(grid.read_cells(cnt, ids[mine]))
        if not (np.array_equal(got_a, ra[mine]) and np.array_equal(got_n, rn[mine])):
            bad.append({"rank": rank, "patch": list(wins[k][0]),
                        "alive_diff": int((got_a != ra[mine]).sum()), "count_diff": int((got_n != rn[mine]).sum())})
    ca, cn = grid.checksum(cur), grid.checksum(cnt)
    parts = allgather({"bad": bad, "alive": ca, "count": cn, "cells": int(sum(int(m.sum()) for _, m, _, _ in expect))})
    got = [sum(p["alive"][0] for p in parts), sum(p["alive"][1] for p in parts) & M64,
           sum(p["count"][0] for p in parts), sum(p["count"][1] for p in parts) & M64]
    mism = [b for p in parts for b in p["bad"]]
    cells = sum(p["cells"] for p in parts)
    ok = not mism and got == sums and cells == sum(ids.size for ids, _, _, _ in expect)
    return {"patches": len(wins), "window_cells": cells, "steps": CHECK_K,
            "corners": [list(c) for c, _ in wins],
            "checker": "bench.gol_box (numpy B3/S23 over 26 neighbors; tests/test_bench_check.py pins it "
                       "to the oracle)",
            "windows_bit_exact": not mism, "checksum_equal": got == sums, "bit_exact": ok,
            "mismatches": mism[:8]}


class Watchdog:
    """Ends the process (exit 3) with a message naming the rank and the phase
    if the phase does not finish in time: a stalled ncclCommInitRank or first
    exchange fails fast instead of holding the job."""

    def __init__(self, rank: int, what: str, seconds: float):
        self.rank, self.what, self.seconds = rank, what, seconds

    def _fire(self):
        os.write(2, f"bench.py: rank {self.rank} stalled in {self.what} for {self.seconds:.0f} s\n".encode())
        os._exit(3)

    def __enter__(self):
        import threading
        self.t = threading.Timer(self.seconds, self._fire)
        self.t.daemon = True
        self.t.start()
        return self

    def __exit__(self, *exc):
        self.t.cancel()
        return False


def poisson3d_leaves():
    """tests/poisson/poisson3d.cpp:158-178's grid: 8^3, the 2x2x2 block around
    (pi, pi/2, 4 pi) refined, the 24 level-0 cells face-adjacent to it refined
    by the reference's induce rule (dccrg.hpp:9730-9800), and the 8 level-1
    cells touching the centre refined again: 792 leaves (max_ref_lvl 2).
    tests/test_bench_inputs.py checks this against the oracle's construction.
    Returns (ids, indices in level-2 units, levels)."""
    N0 = 512
    first = [1, 1 + N0, 1 + 9 * N0]
    blk = {(x, y, z) for x in (3, 4) for y in (3, 4) for z in (3, 4)}
    ref0 = set(blk)
    for (x, y, z) in blk:
        for d in ((1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)):
            ref0.add(((x + d[0]) % 8, (y + d[1]) % 8, (z + d[2]) % 8))
    ids, idx, lvl = [], [], []
    for z in range(8):
        for y in range(8):
            for x in range(8):
                if (x, y, z) not in ref0:
                    ids.append(first[0] + x + 8 * y + 64 * z)
                    idx.append((4 * x, 4 * y, 4 * z))
                    lvl.append(0)
                    continue
                for dz in (0, 1):
                    for dy in (0, 1):
                        for dx in (0, 1):
                            x1, y1, z1 = 2 * x + dx, 2 * y + dy, 2 * z + dz
                            if (x1 in (7, 8) and y1 in (7, 8) and z1 in (7, 8)):
                                for ez in (0, 1):
                                    for ey in (0, 1):
                                        for ex in (0, 1):
                                            x2, y2, z2 = 2 * x1 + ex, 2 * y1 + ey, 2 * z1 + ez
                                            ids.append(first[2] + x2 + 32 * y2 + 1024 * z2)
                                            idx.append((x2, y2, z2))
                                            lvl.append(2)
                            else:
                                ids.append(first[1] + x1 + 16 * y1 + 256 * z1)
                                idx.append((2 * x1, 2 * y1, 2 * z1))
                                lvl.append(1)
    order = np.argsort(ids)
    return (np.array(ids, dtype=np.uint64)[order], np.array(idx, dtype=np.float64)[order],
            np.array(lvl)[order])


def secondary_host_heavy(ctx, D):
    """configs[2] (advection: the solver, then the loop adapting every step)
    and configs[4] (Poisson), whose host-side work (refinement decisions,
    solver control) is sensitive to the process state: measured first, in a
    fresh process as the reference runs each program, before the headline
    grid's ~100 GB of fields and the RCCL contexts of the other lines."""
    out = {}
    # configs[2]: tests/advection/2d.cpp, 400x400x1, max_ref_lvl 2, hood 0:
    # the program's own pre-refinement, then (a) the solver alone on that
    # mixed-level grid and (b) the full loop with adaptation every step
    # (adapt_n = 1: solve, check_for_adaptation, apply, adapt_grid, dt)
    from dccrg_amd import advection as A
    rel, thr, sens, cfl, M = 0.025, 0.25, 0.5, 0.5, 2
    t0 = time.perf_counter()
    g = (D.Dccrg().set_initial_length((400, 400, 1)).set_maximum_refinement_level(M)
         .set_periodic(True, True, False).set_neighborhood_length(0).initialize(ctx))
    g.add_advection_fields()
    geom = A.geometry_2d(g)
    A.initialize(g, geom)
    for _ in range(M):
        A.adapt_grid(g, geom, *A.check_for_adaptation(g, rel / M, thr, sens))
        A.initialize(g, geom)
    t_pre = time.perf_counter() - t0
    nl = g.n_local
    dt_adv = g.max_time_step()
    g.advect_step(cfl * dt_adv)
    ctx.synchronize()
    steps = 50
    t0 = time.perf_counter()
    for _ in range(steps):
        g.advect_step(cfl * dt_adv)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    out["advection"] = {"workload": "configs[2] tests/advection/2d.cpp 400x400x1, max_ref_lvl 2, neighborhood 0, "
                                    f"fp64: solver steps on the pre-refined grid ({nl} leaf cells)",
                        "value": nl * steps / dt, "unit": "cell-steps/s", "steps": steps,
                        "achieved_GBs": 72 * nl * steps / dt / 1e9,
                        "frac": 72 * nl * steps / dt / 1e9 / HBM_PEAK_GBS, "bytes_per_cell_step": 72,
                        "prerefine_s": t_pre}
    # (b) adaptive loop
    g.update_copies_of_remote_neighbors(fields=list(A.ALL))
    steps, cells_steps = 20, 0
    t_adapt = 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        cells_steps += g.n_local
        g.update_copies_of_remote_neighbors(fields=["density"])
        # check_for_adaptation + the adapter's requests, the sets kept on the
        # device (A.check_and_request; the same request state as 2d.cpp's
        # check, then adapt_grid's request loops)
        A.check_and_request(g, rel / M, thr, sens)
        g.advect_step(cfl * dt_adv)
        ta = time.perf_counter()
        A.finish_adaptation(g, geom)
        dt_adv = g.max_time_step()
        t_adapt += time.perf_counter() - ta
    ctx.synchronize()
    dt = time.perf_counter() - t0
    out["advection_adaptive"] = {"workload": "configs[2] tests/advection/2d.cpp loop with adapt_n = 1 "
                                             "(refine/unrefine and device rebuild every step)",
                                 "value": cells_steps / dt, "unit": "cell-steps/s", "steps": steps,
                                 "ms_per_step": dt * 1e3 / steps, "adapt_ms_per_step": t_adapt * 1e3 / steps,
                                 "leaf_cells_end": g.n_local}
    g.close()

    # configs[4] (Poisson part): poisson3d's 792-leaf grid on one GPU
    pl, pidx, plv = poisson3d_leaves()
    L0 = np.array([2 * np.pi / 8, np.pi / 8, 8 * np.pi / 8])
    g = (D.Dccrg().set_initial_length((8, 8, 8)).set_maximum_refinement_level(2)
         .set_periodic(True, True, True).set_neighborhood_length(0).initialize(ctx, leaves=pl))
    for f in ("rhs", "solution", "length_x", "length_y", "length_z"):
        g.add_field(f, np.float64)
    pln = L0[None, :] / (2.0 ** plv)[:, None]
    pc = pidx * (L0 / 4)[None, :] + pln / 2
    g.write_local("rhs", -(81.0 / 16.0) * np.sin(pc[:, 0]) * np.cos(2 * pc[:, 1]) * np.sin(pc[:, 2] / 4))
    for k, a in enumerate(("length_x", "length_y", "length_z")):
        g.write_local(a, pln[:, k])
    s = D.PoissonSolve(g)
    g.write_local("solution", np.zeros(len(pl)))
    s.solve(pl)
    reps = 20
    t0 = time.perf_counter()
    its = 0
    for _ in range(reps):
        g.write_local("solution", np.zeros(len(pl)))
        it_, _ = s.solve(pl, cache_is_up_to_date=True)
        its += it_
    dt = time.perf_counter() - t0
    out["poisson"] = {"workload": "configs[4] tests/poisson/poisson3d 8^3 refined twice (792 leaves), BiCG, "
                                  "1 GPU", "solve_ms": dt * 1e3 / reps, "iterations_per_s": its / dt,
                      "iterations_per_solve": its / reps,
                      "note": "792 cells: one workgroup runs the whole solve (k_solo_lds, LDS-resident), latency bound"}
    s.close()
    g.close()

    return out


def secondary(ctx, torch, D):
    """One line per other BASELINE config (N = 1 only): the 2-D game of life
    (configs[1]), advection on a 2-level refined grid (configs[2]), the
    Poisson solve of configs[4] and the mapping kernel."""
    out = {}
    dev = torch.device("cuda", ctx.device)
    # the N > 1 step structure on one GPU: the 2048^3 slab's periodic images
    # travel as RCCL send/recv to the rank itself (pack, grouped send/recv,
    # unpack) while the inner slices run, then the outer slices
    rc = D.Context(ctx.device, 0, 1)
    rc.comm_init(D.Context.unique_id())
    rc.route_self_through_rccl(True)
    n = 2048
    g = (D.Dccrg().set_initial_length((n, n, n)).set_neighborhood_length(1)
         .set_maximum_refinement_level(0).set_periodic(False, False, True).initialize(rc))
    for f in ("a", "b", "c"):
        g.add_field(f, np.uint32)
    D.lib().dccrgx_field_init_hash(g._h, g.field_id("a"), 200)
    cur, nxt = "a", "b"
    for _ in range(2):
        g.gol_step(cur, nxt, "c")
        cur, nxt = nxt, cur
    rc.synchronize()
    steps = 10
    g.kernel_timer(reset=1)
    t0 = time.perf_counter()
    for _ in range(steps):
        g.gol_step(cur, nxt, "c")
        cur, nxt = nxt, cur
    rc.synchronize()
    dt = time.perf_counter() - t0
    kms, launches = g.kernel_timer(reset=0)
    g.kernel_timer(reset=-1)
    out["gol3d_rccl_halo"] = {
        "workload": "headline grid with the multi-GPU step structure on one GPU: periodic-z images sent "
                    "through RCCL to the rank itself (2 x 16 MiB per step), inner slices overlapped, "
                    "then outer slices",
        "value": n ** 3 * steps / dt, "unit": "cell-updates/s", "steps": steps,
        "ms_per_step": dt * 1e3 / steps, "kernel_ms_per_step": kms / steps,
        "launches_per_step": launches / steps}
    g.close()
    rc.close()
    # configs[1]: 16384^2, hood 1, periodic x y (scalability.cpp:85)
    n = 16384
    g = (D.Dccrg().set_initial_length((n, n, 1)).set_neighborhood_length(1)
         .set_maximum_refinement_level(0).set_periodic(True, True, False).initialize(ctx))
    for f in ("a", "b", "c"):
        g.add_field(f, np.uint32)
    D.lib().dccrgx_field_init_hash(g._h, g.field_id("a"), 200)
    cur, nxt = "a", "b"
    g.gol_step(cur, nxt, "c")
    ctx.synchronize()
    steps = 50
    g.kernel_timer(reset=1)
    t0 = time.perf_counter()
    for _ in range(steps):
        g.gol_step(cur, nxt, "c")
        cur, nxt = nxt, cur
    ctx.synchronize()
    dt = time.perf_counter() - t0
    kms, _ = g.kernel_timer(reset=0)
    g.kernel_timer(reset=-1)
    ach = BYTES_PER_CELL * n * n * steps / (kms * 1e-3) / 1e9
    out["gol2d"] = {"workload": "configs[1] 2-D game of life 16384x16384, hood 1, periodic x,y",
                    "value": n * n * steps / dt, "unit": "cell-updates/s", "steps": steps,
                    "kernel": "k_gol26_rowv<4, true>", "achieved_GBs": ach, "frac": ach / HBM_PEAK_GBS}
    g.close()

    # mapping kernel: ids -> indices + level, 2048^3 grid at max level 10
    m = D.Mapping((2048, 2048, 2048), 10)
    nid = 1 << 26
    gen = torch.Generator(device=dev).manual_seed(1)
    ids = torch.randint(1, 1 << 62, (nid,), device=dev, dtype=torch.int64, generator=gen)
    m.ids_to_indices(ids)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        m.ids_to_indices(ids)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    out["mapping"] = {"workload": "Mapping::get_indices + get_refinement_level on 2^26 random ids, 2048^3 "
                                  "grid, max_ref_lvl 10", "value": nid / (ms * 1e-3), "unit": "ids/s",
                      "achieved_GBs": 36 * nid / (ms * 1e-3) / 1e9,
                      "frac": 36 * nid / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "bytes_per_id": 36}
    del ids
    out["user_stencil_gol"] = user_stencil_gol(ctx, D)
    out["advection_large"] = advection_large(ctx, D)
    out["mapping_reference_speed_test"] = mapping_speed_test(D, torch, dev)
    out["neighbor_lists"] = neighbor_lists(ctx, D, torch)
    return out


def user_stencil_gol(ctx, D):
    """The reference's game of life written as a user functor over
    include/dccrgx_stencil.hpp (examples/user_stencil.hip: count over
    cell.neighbors_of in iteration order, then B3/S23 -- examples/
    game_of_life.cpp:54-79) on the headline grid, beside the library's own
    kernel from the same state: the states and counts must agree.  Two forms:
    for_each_cell_staged (the alive values staged through LDS and a register
    window; the boundary shell walked in separate launches) and for_each_cell
    (every neighbor read through its slot)."""
    import ctypes as C
    L = C.CDLL(US_LIB)
    L.us_gol.argtypes = [C.c_void_p] + [C.c_int32] * 5
    L.us_gol_staged.argtypes = [C.c_void_p] + [C.c_int32] * 6
    n = 2048
    g = (D.Dccrg().set_initial_length((n, n, n)).set_neighborhood_length(1)
         .set_maximum_refinement_level(0).set_periodic(False, False, True).initialize(ctx))
    try:
        for f in ("a", "b", "n", "c", "d"):
            g.add_field(f, np.uint32)
        D.lib().dccrgx_field_init_hash(g._h, g.field_id("a"), 200)
        hood = D.DEFAULT_NEIGHBORHOOD_ID
        f = g.field_id
        g.gol_step("a", "c", "d")  # the library's step from the same state
        ctx.synchronize()
        ref = (g.checksum("c"), g.checksum("d"))

        def run(step, steps):
            # one step a -> b (counts n) checked against the library's, then
            # `steps` timed steps
            if step("a", "b") != 0:
                raise RuntimeError("user stencil launch failed")
            ctx.synchronize()
            same = (g.checksum("b"), g.checksum("n")) == ref
            cur, nxt = "b", "a"
            t0 = time.perf_counter()
            for _ in range(steps):
                step(cur, nxt)
                cur, nxt = nxt, cur
            ctx.synchronize()
            dt = time.perf_counter() - t0
            D.lib().dccrgx_field_init_hash(g._h, g.field_id("a"), 200)  # back to the initial state
            ach = BYTES_PER_CELL * n ** 3 * steps / dt / 1e9
            return {"value": n ** 3 * steps / dt, "unit": "cell-updates/s", "steps": steps,
                    "ms_per_step": dt * 1e3 / steps, "achieved_GBs": ach, "frac": ach / HBM_PEAK_GBS,
                    "equals_library_step": same}

        staged = run(lambda a, b: L.us_gol_staged(g._h, hood, f(a), f(b), f("n"), 0, 1), 10)
        one_stream = run(lambda a, b: L.us_gol_staged(g._h, hood, f(a), f(b), f("n"), 0, 2), 10)
        walk = run(lambda a, b: L.us_gol(g._h, hood, f(a), f(b), f("n"), 0), 3)
        staged["workload"] = ("headline grid (2048^3, hood 1, periodic z) stepped by the game of life written as a "
                              "device user functor over staged values (include/dccrgx_stencil.hpp "
                              "for_each_cell_staged, examples/user_stencil.hip us_gol_staged): the staged kernel "
                              "(LDS-DMA planes; the interior and the edge columns), the edge rows' march and the "
                              "wrap slices on a second stream, every launch of one step")
        walk["workload"] = ("the same functor reading every neighbor through its slot (for_each_cell, "
                            "examples/user_stencil.hip us_gol)")
        staged["walk"] = walk
        one_stream["workload"] = "the staged launches with the edge walks on the caller's stream (no side stream)"
        staged["one_stream"] = one_stream
        return staged
    finally:
        g.close()


def advection_large(ctx, D):
    """configs[2]'s solver (tests/advection/2d.cpp, max_ref_lvl 2, hood 0,
    fp64) on a 16x larger box, 1600 x 1600 pre-refined by the same rules at a
    threshold scaled to the finer density differences (0.006): ~3.5 M leaves,
    where the face-flux kernel is bandwidth- rather than launch-bound.  The
    time is the solver steps only."""
    from dccrg_amd import advection as A
    rel, thr, sens, cfl, M = 0.006, 0.25, 0.5, 0.5, 2
    g = (D.Dccrg().set_initial_length((1600, 1600, 1)).set_maximum_refinement_level(M)
         .set_periodic(True, True, False).set_neighborhood_length(0).initialize(ctx))
    g.add_advection_fields()
    geom = A.geometry_2d(g)
    A.initialize(g, geom)
    for _ in range(M):
        A.adapt_grid(g, geom, *A.check_for_adaptation(g, rel / M, thr, sens))
        A.initialize(g, geom)
    nl = g.n_local
    dt_adv = g.max_time_step()
    for _ in range(2):
        g.advect_step(cfl * dt_adv)
    ctx.synchronize()
    steps = 50
    t0 = time.perf_counter()
    for _ in range(steps):
        g.advect_step(cfl * dt_adv)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    g.close()
    return {"workload": f"tests/advection/2d.cpp solver on 1600x1600x1 pre-refined to {nl} leaf cells "
                        "(max_ref_lvl 2, hood 0, fp64, threshold 0.006)",
            "value": nl * steps / dt, "unit": "cell-steps/s", "steps": steps, "us_per_step": dt * 1e6 / steps,
            "achieved_GBs": 72 * nl * steps / dt / 1e9, "frac": 72 * nl * steps / dt / 1e9 / HBM_PEAK_GBS,
            "bytes_per_cell_step": 72}


def mapping_speed_test(D, torch, dev):
    """tests/geometry/cartesian_grid_speed.cpp's workload: ids 1..1e8 of a
    100x200x300 grid at its maximum refinement level (13).  The reference's
    own program (built where it lies into oracle/_ref/geometry_speed; one
    core, clock()) times get_length and get_center over them; the device
    maps the same ids to indices + level (dccrgx_map_ids_to_indices, what
    get_center spends its time on)."""
    out = {"workload": "Mapping ids 1..1e8 of 100x200x300 at max_ref_lvl 13 (cartesian_grid_speed.cpp)"}
    m = D.Mapping((100, 200, 300), -1)
    n = 100_000_000
    ids = torch.arange(1, n + 1, dtype=torch.int64, device=dev)
    m.ids_to_indices(ids)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        m.ids_to_indices(ids)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    out["device_ids_per_s"] = n / (ms * 1e-3)
    del ids
    exe = os.path.join(ROOT, "oracle", "_ref", "geometry_speed")
    if os.path.exists(exe):
        import re
        import subprocess
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
        t = [float(x) for x in re.findall(r"time for 1e\+08 cells: ([0-9.eE+-]+) s", r.stdout)]
        if len(t) == 2:
            out["reference_cpu"] = {"kind": "reference", "cores": 1,
                                    "get_length_ids_per_s": 1e8 / t[0], "get_center_ids_per_s": 1e8 / t[1]}
            out["device_over_reference_get_center"] = out["device_ids_per_s"] / (1e8 / t[1])
    return out


def neighbor_lists(ctx, D, torch):
    """SURVEY 8(d) 'neighbor build': batched get_neighbors_of (dccrgx_neighbors_of:
    row counts, scan, fill pass) on the device, one call per query with the
    capacity known (`ms`); `ms_with_sizing_call` adds the sizing call of the
    two-call protocol.  Output bytes = entries x 20 B (u64 id + 3 x i32
    offset) + 8 B of row pointer per cell.
    (a) uniform 1024^3 grid, hood 1, periodic z: the first 2^24 cells
        (closed-form lists, dccrg.hpp:4375-4716 on a level-0 grid);
    (b) mixed levels: 128^3 with 5 % of the cells refined once (2.8 M
        leaves), hood 1: lists of every leaf by the face-graph walk kernel
        (k_ex_nof), plus the wall time of initialize() for that grid (hash,
        face graph, lists of every leaf, per-rank lists, stencil rows)."""
    dev = torch.device("cuda", ctx.device)
    X = D._capi
    out = {}

    def query(g, cells, reps):
        q = cells.numel()
        row = torch.zeros(q + 1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)
        X.check(D.lib().dccrgx_neighbors_of(g._h, X.DEFAULT_NEIGHBORHOOD_ID, cells.data_ptr(), q, row.data_ptr(),
                                            None, None, 0, None))
        total = int(row[-1].item())
        ids = torch.empty(total, dtype=torch.int64, device=dev)
        off = torch.empty((total, 3), dtype=torch.int32, device=dev)

        def fill():  # one call: rows and lists (the capacity is known)
            X.check(D.lib().dccrgx_neighbors_of(g._h, X.DEFAULT_NEIGHBORHOOD_ID, cells.data_ptr(), q,
                                                row.data_ptr(), ids.data_ptr(), off.data_ptr(), total, None))

        def sized():  # the two-call protocol: size, then fill
            X.check(D.lib().dccrgx_neighbors_of(g._h, X.DEFAULT_NEIGHBORHOOD_ID, cells.data_ptr(), q,
                                                row.data_ptr(), None, None, 0, None))
            fill()

        def timed(fn):
            fn()
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            ctx.synchronize()
            return (time.perf_counter() - t0) / reps
        dt, dt2 = timed(fill), timed(sized)
        byt = 20 * total + 8 * (q + 1)
        del ids, off, row
        return {"cells": q, "entries": total, "ms": dt * 1e3, "cells_per_s": q / dt, "output_GBs": byt / dt / 1e9,
                "ms_with_sizing_call": dt2 * 1e3}

    n = 1024
    g = (D.Dccrg().set_initial_length((n, n, n)).set_neighborhood_length(1)
         .set_maximum_refinement_level(0).set_periodic(False, False, True).initialize(ctx))
    out["uniform"] = {"workload": "get_neighbors_of of the first 2^24 cells of a 1024^3 grid, hood 1, periodic z",
                      **query(g, torch.arange(1, (1 << 24) + 1, dtype=torch.int64, device=dev), 5)}
    g.close()

    L0 = 128
    n0 = L0 ** 3
    rng = np.random.default_rng(5)
    ref = np.sort(rng.choice(np.arange(1, n0 + 1, dtype=np.int64), size=n0 // 20, replace=False))
    keep = np.setdiff1d(np.arange(1, n0 + 1, dtype=np.int64), ref, assume_unique=True)
    x, y, z = (ref - 1) % L0, ((ref - 1) // L0) % L0, (ref - 1) // (L0 * L0)
    kids = [n0 + 1 + (2 * x + dx) + (2 * y + dy) * 2 * L0 + (2 * z + dz) * 4 * L0 * L0
            for dz in (0, 1) for dy in (0, 1) for dx in (0, 1)]
    leaves = np.sort(np.concatenate([keep] + kids)).astype(np.uint64)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    g = (D.Dccrg().set_initial_length((L0, L0, L0)).set_neighborhood_length(1)
         .set_maximum_refinement_level(1).set_periodic(True, True, True).initialize(ctx, leaves=leaves))
    ctx.synchronize()
    t_init = time.perf_counter() - t0
    cells = torch.from_numpy(leaves.view(np.int64)).to(dev)
    out["mixed_levels"] = {"workload": f"get_neighbors_of of every leaf of a 128^3 grid with 5 % of the cells "
                                       f"refined once ({leaves.size} leaves), hood 1, periodic",
                           "initialize_s": t_init, "initialize_leaves_per_s": leaves.size / t_init,
                           **query(g, cells, 3)}
    # get_neighbors_to of every leaf (dccrgx_neighbors_to: rows of the stored
    # transpose, ids looked up from leaf indices); 8 B per entry + 8 B per row
    q = cells.numel()
    row = torch.zeros(q + 1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    X.check(D.lib().dccrgx_neighbors_to(g._h, X.DEFAULT_NEIGHBORHOOD_ID, cells.data_ptr(), q, row.data_ptr(), None,
                                        0, None))
    total = int(row[-1].item())
    ids = torch.empty(total, dtype=torch.int64, device=dev)

    def to_query():
        X.check(D.lib().dccrgx_neighbors_to(g._h, X.DEFAULT_NEIGHBORHOOD_ID, cells.data_ptr(), q, row.data_ptr(),
                                            ids.data_ptr(), total, None))
    to_query()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        to_query()
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / 3
    out["mixed_levels_to"] = {"workload": "get_neighbors_to of every leaf of the same grid", "cells": q,
                              "entries": total, "ms": dt * 1e3, "output_GBs": (8 * total + 8 * (q + 1)) / dt / 1e9}
    del ids, row
    g.close()
    return out


def halo_payload(ctx, D, world, barrier, reduce_max, shared_gpu=False):
    """tests/scalability/scalability.cpp:170-191 on the device: cells carry
    data_size opaque bytes (its Cell::data, :39-57), each step is
    start_remote_neighbor_copy_updates, wait receives, wait sends around an
    empty "solve" (the busy-wait :79-99 has no device meaning).  A z-slab of
    2048 x 2048 x 8 cells per rank, hood 1, periodic z: at N > 1 the two
    boundary planes go to the ring neighbours through RCCL over xGMI; at N = 1
    the rank's own periodic images go through RCCL to itself."""
    own = None
    c = ctx
    if world == 1:
        own = c = D.Context(ctx.device, 0, 1)
        own.comm_init(D.Context.unique_id())
        own.route_self_through_rccl(True)
    n, depth, steps = 2048, 8, 10
    rows = []
    for ds in (1, 8, 72):
        g = (D.Dccrg().set_initial_length((n, n, depth * world)).set_neighborhood_length(1)
             .set_maximum_refinement_level(0).set_periodic(False, False, True).initialize(c))
        g.add_field("data", np.dtype((np.uint8, ds)))
        ns = g.get_number_of_update_send_cells()
        nr = g.get_number_of_update_receive_cells()
        for _ in range(2):
            g.update_copies_of_remote_neighbors(fields=["data"])
        c.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            g.start_remote_neighbor_copy_updates(fields=["data"])
            g.wait_remote_neighbor_copy_update_receives()
            g.wait_remote_neighbor_copy_update_sends()
        c.synchronize()
        barrier()
        dt = reduce_max(time.perf_counter() - t0)
        rows.append({"data_size": ds, "send_cells_per_rank": ns, "receive_cells_per_rank": nr,
                     "bytes_sent_per_step": ns * ds * world, "ms_per_update": dt * 1e3 / steps,
                     "GBs_per_rank": ns * ds * steps / dt / 1e9})
        g.close()
    # variable-size cells (tests/variable_data_size): cell id holds
    # splitmix64(id) % 17 doubles (mean 8, 64 B); receivers size their ghosts
    # with the same rule, as the reference's receivers must know the sizes
    g = (D.Dccrg().set_initial_length((n, n, depth * world)).set_neighborhood_length(1)
         .set_maximum_refinement_level(0).set_periodic(False, False, True).initialize(c))
    g.add_variable_field("var", np.float64)
    rank, lz = c.rank, depth * world

    def plane(z):
        return (z % lz) * n * n + 1 + np.arange(n * n, dtype=np.uint64)

    def counts(ids):
        x = ids + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return ((x ^ (x >> np.uint64(31))) % np.uint64(17)).astype(np.uint32)

    with np.errstate(over="ignore"):
        send = np.concatenate([plane(rank * depth), plane((rank + 1) * depth - 1)])
        ghost = np.concatenate([plane(rank * depth - 1), plane((rank + 1) * depth)])
        g.resize("var", send, counts(send))
        g.resize("var", ghost, counts(ghost))
        sent = int(counts(send).astype(np.int64).sum()) * 8
    for _ in range(2):  # the first update builds the cached segment plans
        g.update_copies_of_remote_neighbors(fields=["var"])
    c.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.start_remote_neighbor_copy_updates(fields=["var"])
        g.wait_remote_neighbor_copy_update_receives()
        g.wait_remote_neighbor_copy_update_sends()
    c.synchronize()
    barrier()
    dt = reduce_max(time.perf_counter() - t0)
    rows.append({"data_size": "variable: splitmix64(id) % 17 f64 per cell (mean 64 B)",
                 "send_cells_per_rank": int(send.size), "receive_cells_per_rank": int(ghost.size),
                 "bytes_sent_per_step": sent * world, "ms_per_update": dt * 1e3 / steps,
                 "GBs_per_rank": sent * steps / dt / 1e9})
    g.close()
    if own is not None:
        own.close()
    return {"workload": "tests/scalability/scalability.cpp byte payloads (and variable-size cells as in "
                        "tests/variable_data_size), 2048x2048x8 z-slab per rank, hood 1, "
                        "periodic z, start / wait receives / wait sends, empty solve"
                        + (" (N = 1: own periodic images through RCCL)" if world == 1 else
                           ", host-staged transport (ranks share a GPU)" if shared_gpu else ", RCCL over xGMI"),
            "steps": steps, "sizes": rows}


def launch_ranks(n: int) -> int:
    """Run this script as n ranks on this node (the driver's own command:
    torch.distributed.run --nnodes=1 --nproc-per-node n --master-addr
    127.0.0.1), with the same arguments; returns the launcher's exit code.
    Output of the ranks (rank 0 prints the JSON line) goes to this process's
    stdout."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    # torch.distributed.run's parser takes "--n" for an abbreviation of its own options
    args = ["--cells-per-axis" + a[3:] if a == "--n" or a.startswith("--n=") else a for a in sys.argv[1:]]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + args
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", "--cells-per-axis", dest="n", type=int, default=2048, help="cells per axis per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the other configs' lines (N = 1)")
    ap.add_argument("--no-halo-payload", action="store_true", help="skip the byte-payload halo line")
    ap.add_argument("--no-check", action="store_true", help="skip the self-check after the timed loop (profiling)")
    ap.add_argument("--test-corrupt-ghost", action="store_true",
                    help="tests: libdccrgx's corrupt_ghost test option (a bad ghost cell after every exchange); "
                         "the self-check must fail")
    ap.add_argument("--stall-timeout", type=float, default=180.0,
                    help="seconds before a rank stuck in RCCL init or the first exchange ends the run (exit 3)")
    ap.add_argument("--dry-run", action="store_true",
                    help="print each rank's RANK / LOCAL_RANK / WORLD_SIZE as JSON and stop before any GPU call")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # started without a launcher: one process per GPU, spawned here before
        # this process touches the GPU; rank 0's JSON line is relayed
        raise SystemExit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        line = json.dumps({"rank": rank, "local_rank": local_rank, "world_size": world, "gpus": args.gpus, "n": args.n,
                           "master": f"{os.environ.get('MASTER_ADDR', '')}:{os.environ.get('MASTER_PORT', '')}"})
        os.write(1, (line + "\n").encode())  # one write: ranks share the launcher's stdout pipe
        return
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist
    import dccrg_amd as D

    ndev = torch.cuda.device_count()
    device = local_rank % max(ndev, 1)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    if args.test_corrupt_ghost:
        from dccrg_amd.grid import set_test_option
        set_test_option("corrupt_ghost", 1)
    ctx = D.Context(device, rank, world)
    # ranks on the same physical GPU (a rehearsal on one GPU): RCCL refuses
    # that.  Decided from the devices' PCI ids, so a launcher that makes one
    # GPU visible per process still gets RCCL between distinct GPUs.
    shared_gpu = False
    if world > 1:
        pr = torch.cuda.get_device_properties(device)
        ids = [None] * world
        dist.all_gather_object(ids, (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id))
        shared_gpu = len(set(ids)) < world
    if world > 1 and not shared_gpu:
        uid = [D.Context.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        with Watchdog(rank, "ncclCommInitRank", args.stall_timeout):
            ctx.comm_init(uid[0])
    elif world > 1:  # halos through the library's host-staged transport over gloo
        from dccrg_amd.transport import TorchDistTransport
        TorchDistTransport().attach(ctx)

    early = {}
    if rank == 0 and world == 1 and not args.no_secondary:
        early = secondary_host_heavy(ctx, D)

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
    for i in range(args.warmup):
        if i == 0:
            with Watchdog(rank, "the first halo exchange (warm-up step 1)", args.stall_timeout):
                grid.gol_step(cur, nxt, "count")
                barrier()
        else:
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
                        "neighbors), periodic z, block (z-slab) partition, halo over "
                        + ("the host-staged transport (ranks share a GPU)" if shared_gpu else "RCCL"),
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
            "kernel": "dccrgx::k_gol26v<8, 4, true, 1, false>",
            "kernel_ms_per_step": kern_ms / args.steps,
            "launches_per_step": launches / max(args.steps, 1),
            "bytes_per_cell": BYTES_PER_CELL,
        },
        "init_s": t_init,
    }
    if launches == args.steps:  # one stencil launch per step (no remote halo split)
        t = pmc_traffic("k_gol26v<8, 4, true", n_local)
        if t:
            line["roofline"]["traffic"] = t[0]
            line["roofline"]["traffic_source"] = t[1]

    def allgather(obj):
        if world == 1:
            return [obj]
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out
    # outside the timing: the same grid, reseeded, checked against the checker
    if not args.no_check:
        with Watchdog(rank, "the self-check", args.stall_timeout + 300):
            line["check"] = check_run(grid, ctx, n, world, rank, ("alive_a", "alive_b", "count"), allgather)
    grid.close()

    def reduce_max(v: float) -> float:
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    if not args.no_halo_payload:  # collective: every rank
        try:
            line["halo_payload"] = halo_payload(ctx, D, world, barrier, reduce_max, shared_gpu)
        except Exception as e:  # the headline line still prints
            line["halo_payload"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_secondary:
        line["secondary"] = {**secondary(ctx, torch, D), **early}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    if "check" in line and not line["check"]["bit_exact"]:
        os.write(2, f"bench.py: rank {rank}: self-check failed: {json.dumps(line['check']['mismatches'])}\n".encode())
        raise SystemExit(4)


if __name__ == "__main__":
    main()
