"""CPU, multi-process (torch.distributed gloo, world size 2 and 3): the halo
protocol the RCCL path relies on.

Per rank (block partition, dccrg.hpp:8098-8145) the per-peer send / receive
lists (dccrg.hpp:8729-8891) must pair up exactly (what rank r sends to q,
in ascending ids, is what q receives from r), so one message per peer and
field matches on both sides (dccrgx_halo_start's grouped send/recv).  A
distributed game of life whose ghosts travel over gloo in that layout must
equal the single-process run.  Uses the oracle's lists as the checker of the
protocol, not the GPU library (no GPU here).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import dccrg_oracle as O

CASES = [((8, 6, 5), (False, False, True), 1), ((7, 9, 1), (True, True, False), 1),
         ((6, 5, 4), (True, True, True), 2), ((10, 4, 3), (False, True, False), 0)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for length, per, hood in CASES:
            g = O.Grid(length, 0, per, hood)
            v = g.rank_view(rank, world)
            # 1. lists pair up: my send list to q == q's receive list from me
            mine = {"send": v["send"], "recv": v["recv"]}
            allv = [None] * world
            dist.all_gather_object(allv, mine)
            for p in range(world):
                assert allv[rank]["send"].get(p, []) == allv[p]["recv"].get(rank, []), (length, rank, p)
            # 2. game of life with gloo halo, field-major messages per peer
            n = int(np.prod(length))
            a = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 300)
            local = np.array(v["local"], dtype=np.int64)
            state = {int(c): int(a[c - 1]) for c in local}
            nof = v["neighbors_of"]
            steps = 4
            for _ in range(steps):
                ghosts = {}
                reqs, rbufs = [], {}
                for p in sorted(set(v["send"]) | set(v["recv"])):
                    if v["send"].get(p):
                        t = torch.tensor([state[c] for c in v["send"][p]], dtype=torch.int32)
                        reqs.append(dist.isend(t, p))
                    if v["recv"].get(p):
                        rbufs[p] = torch.zeros(len(v["recv"][p]), dtype=torch.int32)
                        reqs.append(dist.irecv(rbufs[p], p))
                for r in reqs:
                    r.wait()
                for p, b in rbufs.items():
                    ghosts.update({c: int(x) for c, x in zip(v["recv"][p], b.tolist())})
                cnt = {}
                for c in local:
                    c = int(c)
                    cnt[c] = sum(1 for i, _ in nof[c] if (state.get(i, ghosts.get(i, 0))) != 0)
                for c in local:
                    c = int(c)
                    state[c] = 1 if cnt[c] == 3 else (state[c] if cnt[c] == 2 else 0)
            allstates = [None] * world
            dist.all_gather_object(allstates, state)
            if rank == 0:
                ra, _ = O.gol_reference_run(length, per, hood, a, steps)
                merged = np.zeros(n, dtype=np.uint32)
                for s in allstates:
                    for c, x in s.items():
                        merged[c - 1] = x
                assert np.array_equal(merged, ra), length
        q.put((rank, "ok"))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_halo_protocol_multi_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res
