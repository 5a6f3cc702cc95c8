"""Multi-rank RCCL halo check: run with torch.distributed.run --nproc-per-node P.

Every rank runs the game of life on its slab of a small grid with the real
RCCL halo (dccrgx_gol_step), then rank 0 gathers the states and compares them
with the CPU oracle.  Exit code 0 = bit-exact.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist

    import dccrg_amd as D

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ndev = max(torch.cuda.device_count(), 1)
    ctx = D.Context(int(os.environ.get("LOCAL_RANK", "0")) % ndev, rank, world)
    uid = [D.Context.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    ctx.comm_init(uid[0])
    failures = 0
    cases = [((64, 48, 40), (False, False, True), 1), ((20, 20, 1), (True, True, False), 1),
             ((30, 26, 9), (True, True, True), 2), ((12, 10, 16), (False, True, False), 0)]
    for length, per, hood in cases:
        g = (D.Dccrg().set_initial_length(length).set_periodic(*per).set_neighborhood_length(hood)
             .initialize(ctx))
        for f in ("a", "b", "n"):
            g.add_field(f, np.uint32)
        n = int(np.prod(length))
        ids = g.local_cells()
        from oracle import dccrg_oracle as O
        a0 = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 300)
        g.write_local("a", a0[ids.astype(np.int64) - 1])
        cur, nxt = "a", "b"
        steps = 5
        for _ in range(steps):
            g.gol_step(cur, nxt, "n")
            cur, nxt = nxt, cur
        ctx.synchronize()
        mine = (ids, g.read_local(cur), g.read_local("n"))
        allp = [None] * world
        dist.all_gather_object(allp, mine)
        if rank == 0:
            alive = np.zeros(n, dtype=np.uint32)
            cnt = np.zeros(n, dtype=np.uint32)
            for i, a, c in allp:
                alive[i.astype(np.int64) - 1] = a
                cnt[i.astype(np.int64) - 1] = c
            ra, rc = O.gol_reference_run(length, per, hood, a0, steps)
            ok = np.array_equal(alive, ra) and np.array_equal(cnt, rc)
            print(f"{length} periodic={per} hood={hood} ranks={world}: {'OK' if ok else 'MISMATCH'}",
                  flush=True)
            failures += 0 if ok else 1
        g.close()
    res = [failures]
    dist.broadcast_object_list(res, src=0)
    ctx.close()
    dist.destroy_process_group()
    sys.exit(1 if res[0] else 0)


if __name__ == "__main__":
    main()
