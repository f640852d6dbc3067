"""ctypes binding of libpls.so (include/pls.h).

The product path: every solver call goes through this library.  There is no
CPU fallback -- if libpls.so is missing or no GPU is visible, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_PKG, "libpls.so")

_lib = None


class pls_csr(C.Structure):
    _fields_ = [("nrows", C.c_int64), ("ncols", C.c_int64), ("row_ptr", C.c_void_p),
                ("col", C.c_void_p), ("val", C.c_void_p)]


class pls_result(C.Structure):
    _fields_ = [("its", C.c_int32), ("reason", C.c_int32), ("rnorm", C.c_double),
                ("pc_applies", C.c_int32), ("history_len", C.c_int32)]


class pls_timings(C.Structure):
    _fields_ = [("pc_total", C.c_double), ("pc_solid", C.c_double), ("pc_fluid", C.c_double),
                ("pc_press", C.c_double), ("pc_alloc", C.c_double), ("solver_total", C.c_double),
                ("spmv_total", C.c_double), ("spmv_calls", C.c_int64)]


class pls_synth_spec(C.Structure):
    _fields_ = [("dim", C.c_int32), ("N", C.c_int32), ("seed", C.c_uint64), ("delta", C.c_double)]


EXPORTS = [
    "pls_abi_version", "pls_last_error", "pls_device_count", "pls_set_device", "pls_create",
    "pls_create_synthetic", "pls_setup", "pls_set_option", "pls_create_solver", "pls_destroy",
    "pls_get_sizes", "pls_pc_apply", "pls_solve", "pls_matmult", "pls_solve_device",
    "pls_pc_apply_device", "pls_matmult_device", "pls_synthetic_rhs_device", "pls_device_alloc",
    "pls_device_free", "pls_memcpy_h2d", "pls_memcpy_d2h", "pls_get_result", "pls_get_history",
    "pls_get_timings", "pls_reset_timings", "pls_export_matrix", "pls_get_permutation",
    "pls_bench_spmv", "pls_rccl_unique_id", "pls_comm_create_rccl", "pls_comm_create_callback",
    "pls_comm_destroy", "pls_create_synthetic_dist", "pls_spmv_layout", "pls_update_matrices",
    "pls_bench_copy", "pls_create_dist", "pls_bench_global_sum", "pls_anderson_create",
    "pls_anderson_next", "pls_anderson_destroy", "pls_boomeramg_host_level", "pls_sparse_lu_analyze",
    "pls_get_ksp_stats",
]

ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p)


def lib():
    """Load libpls.so (raises if it is missing: no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libpls.so not found at {LIB_PATH}; build it with "
                           f"`python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int32
    L.pls_last_error.restype = C.c_char_p
    L.pls_device_count.argtypes = [C.POINTER(C.c_int)]
    L.pls_set_device.argtypes = [C.c_int]
    L.pls_create.argtypes = [C.POINTER(pls_csr), C.POINTER(pls_csr), C.POINTER(pls_csr),
                             vp, i64, vp, i64, vp, i64, vp, i64, C.c_char_p, C.POINTER(vp)]
    L.pls_create_synthetic.argtypes = [C.POINTER(pls_synth_spec), C.c_char_p, C.POINTER(vp)]
    for f in ("pls_setup", "pls_create_solver", "pls_destroy", "pls_reset_timings"):
        getattr(L, f).argtypes = [vp]
    L.pls_set_option.argtypes = [vp, C.c_char_p, C.c_char_p]
    L.pls_get_sizes.argtypes = [vp] + [C.POINTER(i64)] * 5
    L.pls_pc_apply.argtypes = [vp, vp, vp]
    L.pls_solve.argtypes = [vp, vp, vp, C.POINTER(pls_result)]
    L.pls_matmult.argtypes = [vp, vp, vp]
    L.pls_solve_device.argtypes = [vp, vp, vp, C.POINTER(pls_result)]
    L.pls_pc_apply_device.argtypes = [vp, vp, vp]
    L.pls_matmult_device.argtypes = [vp, vp, vp]
    L.pls_synthetic_rhs_device.argtypes = [vp, C.c_uint64, vp]
    L.pls_device_alloc.argtypes = [i64, C.POINTER(vp)]
    L.pls_device_free.argtypes = [vp]
    L.pls_memcpy_h2d.argtypes = [vp, vp, i64]
    L.pls_memcpy_d2h.argtypes = [vp, vp, i64]
    L.pls_get_result.argtypes = [vp, C.POINTER(pls_result)]
    L.pls_get_history.argtypes = [vp, vp, i32]
    L.pls_get_timings.argtypes = [vp, C.POINTER(pls_timings)]
    L.pls_get_ksp_stats.argtypes = [vp, C.c_char_p, vp]
    L.pls_export_matrix.argtypes = [vp, C.c_int, C.POINTER(i64), C.POINTER(i64), vp, vp, vp]
    L.pls_get_permutation.argtypes = [vp, vp]
    L.pls_bench_spmv.argtypes = [vp, vp, vp, i32, C.POINTER(C.c_double)]
    L.pls_rccl_unique_id.argtypes = [C.c_char_p]
    L.pls_comm_create_rccl.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(vp)]
    L.pls_comm_create_callback.argtypes = [C.c_int, C.c_int, ALLGATHER_FN, vp, C.POINTER(vp)]
    L.pls_comm_destroy.argtypes = [vp]
    L.pls_update_matrices.argtypes = [vp, C.POINTER(pls_csr), C.POINTER(pls_csr), C.POINTER(pls_csr)]
    L.pls_bench_copy.argtypes = [i64, i32, i32, C.POINTER(C.c_double)]
    L.pls_spmv_layout.argtypes = [vp, C.POINTER(i32), C.POINTER(i64)]
    L.pls_create_synthetic_dist.argtypes = [C.POINTER(pls_synth_spec), C.c_char_p, vp, C.POINTER(vp)]
    L.pls_bench_global_sum.argtypes = [vp, i32, i32, C.POINTER(C.c_double)]
    L.pls_anderson_create.argtypes = [i32, i64, C.POINTER(vp)]
    L.pls_anderson_next.argtypes = [vp, vp]
    L.pls_anderson_destroy.argtypes = [vp]
    L.pls_boomeramg_host_level.argtypes = [C.POINTER(pls_csr), C.c_char_p, C.c_char_p, i64, C.POINTER(i64),
                                           C.POINTER(i64), C.POINTER(i64), C.POINTER(i64), vp, vp, vp, vp]
    L.pls_sparse_lu_analyze.argtypes = [C.POINTER(pls_csr), C.c_char_p, vp, i64, vp, vp, vp]
    L.pls_create_dist.argtypes = [C.POINTER(pls_csr), C.POINTER(pls_csr), C.POINTER(pls_csr), i64,
                                  vp, i64, vp, i64, vp, i64, vp, i64, C.c_char_p, vp, C.POINTER(vp)]
    _lib = L
    return L


def check(rc):
    if rc != 0:
        msg = lib().pls_last_error()
        raise RuntimeError((msg or b"libpls error").decode())


def ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def device_count() -> int:
    n = C.c_int(0)
    check(lib().pls_device_count(C.byref(n)))
    return n.value


class DeviceArray:
    """A float64 device buffer owned through libpls (no torch needed)."""

    def __init__(self, n: int):
        self.n = int(n)
        self.p = C.c_void_p()
        check(lib().pls_device_alloc(max(self.n, 1) * 8, C.byref(self.p)))

    def upload(self, a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        check(lib().pls_memcpy_h2d(self.p, ptr(a), a.size * 8))

    def download(self):
        out = np.empty(self.n, dtype=np.float64)
        check(lib().pls_memcpy_d2h(ptr(out), self.p, self.n * 8))
        return out

    def free(self):
        if self.p:
            lib().pls_device_free(self.p)
            self.p = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def csr_of(M):
    """(indptr int64, indices int32, data float64, nrows, ncols) of a matrix-like.

    Accepts scipy.sparse matrices, petsc4py Mat (``getValuesCSR``), and dolfin
    ``PETScMatrix`` (``.mat()``) -- the objects the reference passes
    (reference lib/Preconditioner.py:284, lib/Solver.py:89,95).
    """
    if hasattr(M, "mat") and callable(M.mat):
        M = M.mat()
    if hasattr(M, "getValuesCSR"):
        ai, aj, av = M.getValuesCSR()
        nr, nc = M.getSize()
        return (np.ascontiguousarray(ai, dtype=np.int64), np.ascontiguousarray(aj, dtype=np.int32),
                np.ascontiguousarray(av, dtype=np.float64), int(nr), int(nc))
    import scipy.sparse as sp
    if sp.issparse(M):
        M = M.tocsr()
        if not M.has_sorted_indices:
            M = M.copy()
            M.sort_indices()
        return (np.ascontiguousarray(M.indptr, dtype=np.int64),
                np.ascontiguousarray(M.indices, dtype=np.int32),
                np.ascontiguousarray(M.data, dtype=np.float64), M.shape[0], M.shape[1])
    raise TypeError(f"unsupported matrix type {type(M)!r}")


def vec_array(v):
    """Writable float64 numpy view/array of a vector-like (numpy, petsc4py Vec, dolfin vector)."""
    if hasattr(v, "vec") and callable(v.vec):
        v = v.vec()
    if hasattr(v, "getArray"):
        return v.getArray()
    return v


def is_array(s):
    if hasattr(s, "getIndices"):
        s = s.getIndices()
    return np.ascontiguousarray(np.asarray(s), dtype=np.int32)
