"""Host-staged halo transport over torch.distributed (dccrgx_host_transport).

RCCL refuses two ranks on one GPU, so processes that share a device cannot
form a communicator.  With this transport set on their contexts, the library
packs each peer's message on the device with the same plans the RCCL path
uses, hands the host copies to ``exchange`` -- point-to-point isend / irecv
of every message of one update over the process group (gloo) -- and unpacks
what arrives; solver scalars go through ``all_reduce``.  This plays the role
of the reference's MPI transfer engine (dccrg.hpp:10726-11209: Isend / Irecv
per peer, then Waitall) for ranks sharing a GPU; on separate GPUs the
library's RCCL path is the data path.
"""
from __future__ import annotations

import ctypes as C
import sys
import traceback

import numpy as np

from . import _capi as X
from ._capi import check, lib


def _host_array(ptr: int, nbytes: int) -> np.ndarray:
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), (nbytes,))


class TorchDistTransport:
    """exchange / allreduce callbacks over the default torch.distributed group."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self._torch, self._dist, self._group = torch, dist, group
        self._c = X.HostTransport_t(None, X.EXCHANGE_FN(self._exchange), X.ALLREDUCE_FN(self._allreduce))

    def _exchange(self, _user, n_send, send_peers, send_bufs, send_bytes, n_recv, recv_peers, recv_bufs,
                  recv_bytes):
        try:
            torch, dist = self._torch, self._dist
            reqs, keep = [], []
            for i in range(n_recv):
                nb = int(recv_bytes[i])
                if nb:
                    t = torch.from_numpy(_host_array(recv_bufs[i], nb))
                    keep.append(t)
                    reqs.append(dist.irecv(t, src=int(recv_peers[i]), group=self._group))
            for i in range(n_send):
                nb = int(send_bytes[i])
                if nb:
                    t = torch.from_numpy(_host_array(send_bufs[i], nb))
                    keep.append(t)
                    reqs.append(dist.isend(t, dst=int(send_peers[i]), group=self._group))
            for r in reqs:
                r.wait()
            return 0
        except Exception:
            traceback.print_exc(file=sys.stderr)
            return 1

    def _allreduce(self, _user, values, n, op):
        try:
            torch, dist = self._torch, self._dist
            a = np.ctypeslib.as_array(values, (n,))
            # every rank's values, combined in rank order on every rank: the
            # result is the same everywhere and does not depend on the
            # collective's internal reduction order
            world = dist.get_world_size(self._group)
            parts = [torch.zeros(n, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(a.copy()), group=self._group)
            if int(op) == 0:
                tot = np.zeros(n)
                for p in parts:
                    tot = tot + p.numpy()
            else:
                stack = np.stack([p.numpy() for p in parts])
                tot = stack.min(axis=0) if int(op) == 1 else stack.max(axis=0)
            a[:] = tot
            return 0
        except Exception:
            traceback.print_exc(file=sys.stderr)
            return 1

    def attach(self, ctx) -> "TorchDistTransport":
        """Set on a dccrg_amd.Context (kept alive by the context)."""
        check(lib().dccrgx_ctx_set_host_transport(ctx._h, C.byref(self._c)))
        ctx._transport = self
        return self
