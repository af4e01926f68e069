"""Multi-rank plumbing of the path (one process per GPU).

The data path's communicator is libafem's own (include/arcanefem_amd.h):
  * ``Communicator`` (core.py): RCCL over xGMI, bootstrapped with an id
    broadcast over torch.distributed -- the production transport;
  * ``HostCommunicator`` (here): the same halo plan and all-reduce points with
    the bytes moved through host memory by torch.distributed (gloo) -- the
    IParallelMng-style transport for hosts where RCCL cannot run (several
    ranks sharing one GPU) and for tests of the distributed path.  Only the
    transport differs: packing / unpacking of the halo (send/recv id lists),
    the CG and its reductions are libafem's.
torch.distributed is the control plane only (process group bootstrap,
barriers); it never touches device memory here.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _capi as C
from ._capi import call


class HostCommunicator:
    """afem_comm_create_host with torch.distributed (gloo) callbacks: the
    reference's IParallelMng::reduce / sendRecv over the ranks of the default
    process group."""

    def __init__(self, ctx, group=None, async_exchange: bool = False):
        import torch
        import torch.distributed as dist

        self._torch, self._dist, self._group = torch, dist, group
        self.rank = dist.get_rank(group)
        self.nranks = dist.get_world_size(group)
        self.errors = []

        def allreduce(user, buf, n):
            try:
                a = np.ctypeslib.as_array(buf, shape=(n,))
                t = torch.from_numpy(a)
                dist.all_reduce(t, group=self._group)
                return 0
            except Exception as e:  # reported through the C status
                self.errors.append(repr(e))
                return 1

        def exchange(user, n_nbr, nbr, send, send_counts, recv, recv_counts):
            try:
                sc = np.ctypeslib.as_array(send_counts, shape=(n_nbr,)).copy()
                rc = np.ctypeslib.as_array(recv_counts, shape=(n_nbr,)).copy()
                sa = np.ctypeslib.as_array(send, shape=(int(sc.sum()),)) if sc.sum() else np.zeros(0)
                ra = np.ctypeslib.as_array(recv, shape=(int(rc.sum()),)) if rc.sum() else np.zeros(0)
                so = np.concatenate([[0], np.cumsum(sc)])
                ro = np.concatenate([[0], np.cumsum(rc)])
                reqs = []
                for i in range(n_nbr):
                    peer = int(nbr[i])
                    if sc[i]:
                        reqs.append(dist.isend(torch.from_numpy(sa[so[i]:so[i + 1]].copy()), peer, group=self._group))
                    if rc[i]:
                        reqs.append(dist.irecv(torch.from_numpy(ra[ro[i]:ro[i + 1]]), peer, group=self._group))
                for r in reqs:
                    r.wait()
                return 0
            except Exception as e:
                self.errors.append(repr(e))
                return 1

        self._fns = (C.ALLREDUCE_FN(allreduce), C.EXCHANGE_FN(exchange))
        self._t = C.HostTransport(None, self._fns[0], self._fns[1])
        h = ctypes.c_void_p()
        call("afem_comm_create_host", ctx.h, self.nranks, self.rank, ctypes.byref(self._t), ctypes.byref(h))
        self.h = h
        if async_exchange:
            # the halo callback then runs on libafem's worker thread while the CG's
            # interior SpMV is on the GPU (afem_comm_host_async)
            call("afem_comm_host_async", self.h, 1)

    def close(self):
        if self.h:
            call("afem_comm_destroy", self.h)
            self.h = None
