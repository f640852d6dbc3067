"""Inner Anderson acceleration (reference lib/AndersonAcceleration.py:6-78).

``AndersonAcceleration(order).get_next_vector(gk)`` as in the reference, on
the device: libpls.so's mixer (``pls_anderson_*``, the same code the block PC
runs for ``inner accel order`` > 0, reference lib/Preconditioner.py:248-249)
keeps the F / X histories in HBM and solves the least squares by Householder
QR (TSQR).  ``gk`` is either a float64 numpy vector -- replaced in place by the
mixed iterate, as the reference's ``self.xk.copy(gk)`` replaces the PETSc Vec
-- or a ``lib._native.DeviceArray`` (mixed on the device, no copies).  The
object is single-rank: under mpirun the handle's inner accel path does the
rank-0 least squares (AndersonAcceleration.py:50-66).
"""
import ctypes as C

import numpy as np

from . import _native as N


class AndersonAcceleration:
    def __init__(self, order):
        self.order = int(order)
        self._obj = None
        self._n = None
        self._buf = None

    def _ensure(self, n):
        if self._obj is None:
            obj = C.c_void_p()
            N.check(N.lib().pls_anderson_create(self.order, n, C.byref(obj)))
            self._obj, self._n = obj, n
        elif n != self._n:
            raise ValueError(f"AndersonAcceleration: vector length {n} != {self._n} of the first call")

    def get_next_vector(self, gk):
        if isinstance(gk, N.DeviceArray):
            self._ensure(gk.n)
            N.check(N.lib().pls_anderson_next(self._obj, gk.p))
            return gk
        if not (isinstance(gk, np.ndarray) and gk.dtype == np.float64 and gk.ndim == 1 and gk.flags.c_contiguous):
            raise TypeError("get_next_vector: gk must be a contiguous 1-D float64 numpy array or a DeviceArray")
        self._ensure(gk.size)
        if self._buf is None:
            self._buf = N.DeviceArray(gk.size)
        self._buf.upload(gk)
        N.check(N.lib().pls_anderson_next(self._obj, self._buf.p))
        gk[:] = self._buf.download()
        return gk

    def destroy(self):
        if self._buf is not None:
            self._buf.free()
            self._buf = None
        if self._obj is not None:
            N.lib().pls_anderson_destroy(self._obj)
            self._obj = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass
