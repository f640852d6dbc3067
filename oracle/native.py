"""ctypes binding of oracle/csrc/oracle.c (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")


def build() -> str:
    """Compile the oracle C kernels (gcc, -ffp-contract=off)."""
    srcs = [os.path.join(_HERE, "csrc", f) for f in ("oracle.c", "cpu_solver.c")]
    if (not os.path.exists(_LIB)) or os.path.getmtime(_LIB) < max(os.path.getmtime(f) for f in srcs):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB):
        build()
    L = C.CDLL(_LIB)
    L.oracle_synth_sizes.argtypes = [C.c_int, C.c_int, C.c_uint64, _i64p]
    L.oracle_synth_offsets.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_int, _i32p]
    L.oracle_synth_rowptr.argtypes = [C.c_int, C.c_int, C.c_uint64, _i64p]
    L.oracle_synth_fill.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_double, C.c_int,
                                    _i64p, _i32p, _f64p]
    L.oracle_synth_rhs.argtypes = [C.c_uint64, C.c_int64, _f64p]
    L.oracle_synth_rhs.restype = None
    L.oracle_synth_is_bc.argtypes = [C.c_uint64, C.c_int64]
    L.oracle_spmv.argtypes = [C.c_int64, _i64p, _i32p, _f64p, _f64p, _f64p, C.c_int]
    L.oracle_spmv.restype = None
    L.oracle_ilu0.argtypes = [C.c_int64, _i64p, _i32p, _f64p, _i64p, _f64p]
    L.oracle_ilu0_solve.argtypes = [C.c_int64, _i64p, _i32p, _f64p, _i64p, _f64p, _f64p, _f64p]
    L.oracle_ilu0_solve.restype = None
    L.oracle_levels.argtypes = [C.c_int64, _i64p, _i32p, C.c_int, _i32p]
    L.oracle_levels.restype = C.c_int64
    L.cpu_gmres_2way.argtypes = [C.c_int64, C.c_int64, _i64p, _i32p, _f64p, _i64p, _i32p, _f64p, C.c_int64,
                                 C.c_int64, C.c_double, C.c_double, C.c_int, _f64p, _f64p, C.POINTER(C.c_int),
                                 _f64p, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.cpu_gmres_2way.restype = C.c_int
    _lib = L
    return L


def csr_arrays(M):
    """(indptr int64, indices int32, data float64), C-contiguous."""
    return (np.ascontiguousarray(M.indptr, dtype=np.int64),
            np.ascontiguousarray(M.indices, dtype=np.int32),
            np.ascontiguousarray(M.data, dtype=np.float64))


def spmv(M, x, nthreads: int = 1) -> np.ndarray:
    rp, ci, v = csr_arrays(M)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty(M.shape[0], dtype=np.float64)
    lib().oracle_spmv(M.shape[0], rp, ci, v, x, y, int(nthreads))
    return y


class ILU0:
    """PETSc ILU(0), natural ordering, on the pattern of ``M`` (sorted columns)."""

    def __init__(self, M):
        M = M.tocsr()
        M.sort_indices()
        self.n = M.shape[0]
        self.rp, self.ci, v = csr_arrays(M)
        self.lu = v.copy()
        self.diag = np.empty(self.n, dtype=np.int64)
        self.dinv = np.zeros(self.n, dtype=np.float64)
        rc = lib().oracle_ilu0(self.n, self.rp, self.ci, self.lu, self.diag, self.dinv)
        if rc < 0:
            raise RuntimeError(f"ILU(0): missing diagonal in row {-rc - 1}")
        if rc > 0:
            raise RuntimeError(f"ILU(0): zero pivot in row {rc - 1}")

    def solve(self, b):
        b = np.ascontiguousarray(b, dtype=np.float64)
        x = np.empty_like(b)
        lib().oracle_ilu0_solve(self.n, self.rp, self.ci, self.lu, self.diag, self.dinv, b, x)
        return x


def levels(M, lower: bool = True):
    rp, ci, _ = csr_arrays(M)
    lvl = np.zeros(M.shape[0], dtype=np.int32)
    nl = lib().oracle_levels(M.shape[0], rp, ci, 0 if lower else 1, lvl)
    return int(nl), lvl


def cpu_gmres_2way(A, P, ns, nb_s, nb_fp, b, rtol=1e-6, atol=1e-8, maxit=100, nthreads=1):
    """C/OpenMP restatement of bench.py's configuration (oracle/csrc/cpu_solver.c):
    right-PC GMRES + 2-way block PC with PREONLY + BJACOBI(ILU(0)) inner solves
    on a field-major system.  Returns (x, its, reason, history, t_setup, t_solve)."""
    Ap, Ai, Av = csr_arrays(A)
    Pp, Pi, Pv = csr_arrays(P)
    b = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros_like(b)
    hist = np.zeros(maxit + 1)
    reason = C.c_int(0)
    ts, tv = C.c_double(0), C.c_double(0)
    its = lib().cpu_gmres_2way(A.shape[0], ns, Ap, Ai, Av, Pp, Pi, Pv, nb_s, nb_fp, rtol, atol, maxit, b, x,
                               C.byref(reason), hist, nthreads, C.byref(ts), C.byref(tv))
    if its < 0:
        raise RuntimeError("cpu_gmres_2way: ILU(0) failed (missing diagonal or zero pivot)")
    return x, its, reason.value, hist[:its + 1], ts.value, tv.value
