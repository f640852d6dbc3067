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
    src = os.path.join(_HERE, "csrc", "oracle.c")
    if (not os.path.exists(_LIB)) or os.path.getmtime(_LIB) < os.path.getmtime(src):
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
