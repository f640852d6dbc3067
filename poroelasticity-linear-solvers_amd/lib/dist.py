"""Communicators of the distributed solve (one process per GPU).

The reference is MPI-parallel through PETSc (``mpirun -np 8 python3 main.py``,
paper-scripts/robustness_2d.sh:29; every Vec/Mat/KSP on COMM_WORLD).  Here a
``Communicator`` wraps a ``pls_comm`` (include/pls.h):

* ``Communicator.rccl()`` -- production: RCCL over xGMI.  Rank 0 makes the
  unique id, ``torch.distributed`` (already initialised by the launcher,
  ``torch.distributed.run``) broadcasts it, every rank joins on its own GPU;
* ``Communicator.host(allgather)`` -- host-staged: libpls calls back into
  Python for every exchange.  ``Communicator.gloo()`` supplies the callback
  from ``torch.distributed`` with a CPU backend, which lets several ranks share
  one GPU (tests) -- RCCL refuses two ranks on one device.

The handle must be destroyed before its communicator (``Handle.synthetic_dist``
keeps a reference so the order holds).
"""
from __future__ import annotations

import ctypes as C
import os

from . import _native as N

_DEFAULT = None


class Communicator:
    def __init__(self, ptr, rank, size, keep=None):
        self.ptr, self.rank, self.size = ptr, rank, size
        self._keep = keep  # the ctypes callback must outlive the communicator

    @classmethod
    def rccl(cls):
        import torch.distributed as td
        rank, size = td.get_rank(), td.get_world_size()
        buf = C.create_string_buffer(128)
        if rank == 0:
            N.check(N.lib().pls_rccl_unique_id(buf))
        obj = [bytes(buf.raw) if rank == 0 else None]
        td.broadcast_object_list(obj, src=0)
        uid = C.create_string_buffer(obj[0], 128)
        out = C.c_void_p()
        N.check(N.lib().pls_comm_create_rccl(uid, rank, size, C.byref(out)))
        return cls(out, rank, size)

    @classmethod
    def host(cls, rank, size, allgather):
        """allgather(bytes_of_this_rank) -> list of ``size`` equal-length bytes."""

        def cb(send, nbytes, recv, user):
            try:
                parts = allgather(C.string_at(send, nbytes))
                blob = b"".join(parts)
                if len(blob) != nbytes * size:
                    return 1
                C.memmove(recv, blob, len(blob))
                return 0
            except Exception:  # noqa: BLE001 -- reported to libpls as failure
                return 1

        fn = N.ALLGATHER_FN(cb)
        out = C.c_void_p()
        N.check(N.lib().pls_comm_create_callback(rank, size, fn, None, C.byref(out)))
        return cls(out, rank, size, keep=fn)

    @classmethod
    def gloo(cls, group=None):
        import torch.distributed as td
        return cls.host(td.get_rank(group), td.get_world_size(group), torch_allgather(group))

    def destroy(self):
        if self.ptr:
            N.lib().pls_comm_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def torch_allgather(group=None):
    """Equal-size byte allgather over a CPU torch.distributed group."""
    import numpy as np
    import torch
    import torch.distributed as td

    def allgather(data: bytes):
        t = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy())
        out = [torch.empty_like(t) for _ in range(td.get_world_size(group))]
        td.all_gather(out, t, group=group)
        return [o.numpy().tobytes() for o in out]

    return allgather


def world():
    """(rank, size) of the torch.distributed job this process belongs to
    ((0, 1) when none is initialised -- the single-process path)."""
    try:
        import torch.distributed as td
        if td.is_available() and td.is_initialized():
            return td.get_rank(), td.get_world_size()
    except ImportError:
        pass
    return 0, 1


def default_communicator():
    """The communicator the facade shards over when the process is one rank of
    a multi-rank job (the reference's ``mpirun -np G``; here torchrun /
    torch.distributed), created once: RCCL on GPU ``LOCAL_RANK`` by default,
    the host-staged gloo communicator when ``PLS_COMM=host`` (ranks sharing a
    GPU).  None on a single rank."""
    global _DEFAULT
    rank, size = world()
    if size <= 1:
        return None
    if _DEFAULT is None:
        if os.environ.get("PLS_COMM", "rccl") == "host":
            _DEFAULT = Communicator.gloo()
        else:
            N.check(N.lib().pls_set_device(int(os.environ.get("LOCAL_RANK", rank))))
            _DEFAULT = Communicator.rccl()
        import atexit
        atexit.register(_release_default)
    return _DEFAULT


def _release_default():
    global _DEFAULT
    if _DEFAULT is not None:
        _DEFAULT.destroy()
        _DEFAULT = None
