"""The multi-rank halo path through the real RCCL communicator on one GPU.

RCCL refuses two ranks on one device, so the N > 1 exchange cannot run on a
one-GPU box as N processes.  Instead a 1-rank communicator carries the rank's
own periodic images as RCCL send/recv to itself
(dccrgx_ctx_route_self_through_rccl): the same peer plans, pack / unpack
kernels, grouped ncclSend / ncclRecv on the communication stream, event
ordering between the streams and the inner / outer overlap split that a
z-slab ring of GPUs uses (scalability3d.cpp:122-166).  Results are compared
bit-exactly with the oracle and with the device-copy path."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import dccrg_amd as D  # noqa: E402
from oracle import dccrg_oracle as O  # noqa: E402


def rccl_ctx():
    c = D.Context(0, 0, 1)
    c.comm_init(D.Context.unique_id())
    c.route_self_through_rccl(True)
    return c


def gol_grid(ctx, L, per, hood):
    g = (D.Dccrg().set_initial_length(L).set_periodic(*per).set_neighborhood_length(hood)
         .set_maximum_refinement_level(0).initialize(ctx))
    for f in ("a", "b", "n"):
        g.add_field(f, np.uint32)
    return g


@pytest.mark.parametrize("L,per,hood", [((40, 24, 16), (True, False, True), 1),
                                        ((17, 13, 11), (True, True, True), 1),
                                        ((20, 18, 12), (False, True, True), 2),
                                        ((64, 48, 1), (True, True, False), 1),
                                        ((9, 8, 7), (True, True, True), 3)])
def test_gol_halo_through_rccl(L, per, hood):
    ctx = rccl_ctx()
    g = gol_grid(ctx, L, per, hood)
    send = g.get_cells_to_send()
    assert list(send) == [0] and g.get_cells_to_receive()[0] == send[0]  # the rank itself is the peer
    n = int(np.prod(L))
    a0 = O.random_alive(np.arange(1, n + 1, dtype=np.uint64), 250)
    steps = 6
    ref_a, ref_n = O.gol_reference_run(L, per, hood, a0, steps)
    g.write_local("a", a0)
    g.kernel_timer(reset=1)
    cur, nxt = "a", "b"
    for _ in range(steps):
        g.gol_step(cur, nxt, "n")
        cur, nxt = nxt, cur
    ctx.synchronize()
    _, launches = g.kernel_timer(reset=0)
    g.kernel_timer(reset=-1)
    assert launches > steps  # inner and outer regions launched separately (overlap split)
    assert np.array_equal(g.read_local(cur), ref_a)
    assert np.array_equal(g.read_local("n"), ref_n)
    g.close()
    ctx.close()


def test_gol_rccl_matches_copy_path_large():
    """A slab of the bench config (2048 x 2048 x 64, periodic z): the RCCL
    path and the device-copy path give identical states after 5 steps."""
    L, per = (2048, 2048, 64), (False, False, True)
    out = []
    for rccl in (True, False):
        ctx = rccl_ctx() if rccl else D.Context(0, 0, 1)
        g = gol_grid(ctx, L, per, 1)
        D.lib().dccrgx_field_init_hash(g._h, g.field_id("a"), 200)
        cur, nxt = "a", "b"
        for _ in range(5):
            g.gol_step(cur, nxt, "n")
            cur, nxt = nxt, cur
        out.append((g.read_local(cur), g.read_local("n")))
        g.close()
        ctx.close()
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])


@pytest.mark.parametrize("L,per,hood", [((32, 24, 1), (True, True, False), 0), ((12, 10, 8), (True, False, True), 1)])
def test_advection_halo_through_rccl(L, per, hood):
    """advect_step's density halo over RCCL: bit-identical to the copy path
    (each cell's face sum is evaluated the same way in either region)."""
    names = ("density", "vx", "vy", "vz", "length_x", "length_y", "length_z")
    res = []
    for rccl in (True, False):
        ctx = rccl_ctx() if rccl else D.Context(0, 0, 1)
        g = (D.Dccrg().set_initial_length(L).set_periodic(*per).set_neighborhood_length(hood)
             .initialize(ctx))
        g.add_advection_fields()
        state = O.advection_initial_state(O.Mapping(L, 0), g.local_cells())
        for name, arr in zip(names, state):
            g.write_local(name, arr)
        g.update_copies_of_remote_neighbors(fields=list(names))
        dt = 0.5 * g.max_time_step()
        for _ in range(8):
            g.advect_step(dt)
        res.append(g.read_local("density"))
        g.close()
        ctx.close()
    assert np.array_equal(res[0], res[1])
