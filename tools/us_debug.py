"""print the device walk of cell 1 of a periodic 10x8x6 grid (debugging)"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dccrg_amd as D  # noqa: E402

L = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "libuser_stencil.so"))
L.us_list.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p]
ctx = D.Context(0, 0, 1)
g = D.Dccrg().set_initial_length((10, 8, 6)).set_periodic(True, True, True).set_neighborhood_length(1).initialize(ctx)
g.add_field("id", np.uint64)
g.write_local("id", g.local_cells())
g.halo_self(fields=["id"])
v = g.stencil_view()
print("view", v.kind, v.n_items, v.n_cells, v.la, v.lb, v.lc, v.lo, v.hi, v.cbase, list(v.s0), list(v.s1), list(v.per),
      list(v.perm), v.scale, list(v.reach))
out = torch.zeros(64 * 4, dtype=torch.int64, device="cuda")
n = torch.zeros(1, dtype=torch.int32, device="cuda")
for cell in (1, 120):
    slot = int(cell - 1 - v.cbase * v.la * v.lb)
    torch.cuda.synchronize()
    assert L.us_list(g._h, D.DEFAULT_NEIGHBORHOOD_ID, g.field_id("id"), slot, out.data_ptr(), 64, n.data_ptr()) == 0
    ctx.synchronize()
    k = int(n.item())
    print(cell, k, out[:4 * k].view(-1, 4).tolist())
g.close()
ctx.close()
