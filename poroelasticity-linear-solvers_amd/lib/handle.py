"""Owning wrapper of a ``pls_handle`` (include/pls.h)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N


def params_to_options(parameters: dict) -> dict:
    """The reference's parameter dict -> ``pls.*`` option keys."""
    keymap = {
        "solver type": "pls.solver_type", "solver atol": "pls.solver_atol", "solver rtol": "pls.solver_rtol",
        "solver maxiter": "pls.solver_maxiter", "solver monitor": "pls.solver_monitor",
        "pc type": "pls.pc_type", "inner ksp type": "pls.inner_ksp_type", "inner pc type": "pls.inner_pc_type",
        "inner rtol": "pls.inner_rtol", "inner atol": "pls.inner_atol", "inner maxiter": "pls.inner_maxiter",
        "inner monitor": "pls.inner_monitor", "inner accel order": "pls.inner_accel_order",
        "AAR order": "pls.aar_order", "AAR p": "pls.aar_p", "AAR omega": "pls.aar_omega", "AAR beta": "pls.aar_beta",
    }
    out = {}
    for k, v in parameters.items():
        if k in keymap:
            if isinstance(v, bool):
                v = "1" if v else "0"
            out[keymap[k]] = str(v).replace(" ", "_")
    return out


def options_text(d: dict) -> bytes:
    lines = []
    for k, v in d.items():
        lines.append(k if v is None else f"{k} {v}")
    return "\n".join(lines).encode()


class Handle:
    def __init__(self, ptr: C.c_void_p):
        self.ptr = ptr
        n, ns, nf, np_, nnz = (C.c_int64() for _ in range(5))
        N.check(N.lib().pls_get_sizes(ptr, C.byref(n), C.byref(ns), C.byref(nf), C.byref(np_), C.byref(nnz)))
        self.n, self.ns, self.nf, self.np, self.nnz_A = n.value, ns.value, nf.value, np_.value, nnz.value

    # ----------------------------------------------------------- creation --
    @classmethod
    def from_csr(cls, A, P, P_diff, is_s, is_f, is_p, bcs_sub_pressure, options: dict):
        keep = []

        def mk(M):
            if M is None:
                return None
            ai, aj, av, nr, nc = N.csr_of(M)
            keep.extend([ai, aj, av])
            return N.pls_csr(nr, nc, ai.ctypes.data, aj.ctypes.data, av.ctypes.data)

        cA, cP, cD = mk(A), mk(P), mk(P_diff)
        is_s, is_f, is_p = N.is_array(is_s), N.is_array(is_f), N.is_array(is_p)
        bcs = np.ascontiguousarray(np.asarray(bcs_sub_pressure if bcs_sub_pressure is not None else [],
                                              dtype=np.int32))
        out = C.c_void_p()
        N.check(N.lib().pls_create(C.byref(cA), C.byref(cP), C.byref(cD) if cD is not None else None,
                                   N.ptr(is_s), is_s.size, N.ptr(is_f), is_f.size, N.ptr(is_p), is_p.size,
                                   N.ptr(bcs), bcs.size, options_text(options), C.byref(out)))
        return cls(out)

    @classmethod
    def from_csr_dist(cls, A, P, P_diff, is_s, is_f, is_p, bcs_sub_pressure, options: dict, comm, row_start=None):
        """This rank's share of a caller-assembled system (pls_create_dist):
        A, P, P_diff = the rank's rows (global columns), is_* = the global
        indices of the dofs it owns, bcs_sub_pressure = positions inside its p
        sub-vector.  ``row_start`` (the rank's first global row) defaults to
        the smallest owned index.  Collective over ``comm``; host vectors are
        the rank's rows in the caller's order."""
        keep = []
        is_s, is_f, is_p = N.is_array(is_s), N.is_array(is_f), N.is_array(is_p)
        nloc = is_s.size + is_f.size + is_p.size
        if row_start is None:
            row_start = int(min(a.min() for a in (is_s, is_f, is_p) if a.size)) if nloc else 0

        def mk(M):
            if M is None:
                return None
            ai, aj, av, _, nc = N.csr_of(M)
            keep.extend([ai, aj, av])
            return N.pls_csr(ai.size - 1, nc, ai.ctypes.data, aj.ctypes.data, av.ctypes.data)

        cA, cP, cD = mk(A), mk(P), mk(P_diff)
        bcs = np.ascontiguousarray(np.asarray(bcs_sub_pressure if bcs_sub_pressure is not None else [],
                                              dtype=np.int32))
        out = C.c_void_p()
        N.check(N.lib().pls_create_dist(C.byref(cA), C.byref(cP), C.byref(cD) if cD is not None else None,
                                        int(row_start), N.ptr(is_s), is_s.size, N.ptr(is_f), is_f.size,
                                        N.ptr(is_p), is_p.size, N.ptr(bcs), bcs.size, options_text(options),
                                        comm.ptr, C.byref(out)))
        h = cls(out)
        h._comm = comm
        return h

    @classmethod
    def synthetic(cls, dim, Nel, seed, delta, options: dict):
        spec = N.pls_synth_spec(int(dim), int(Nel), int(seed), float(delta))
        out = C.c_void_p()
        N.check(N.lib().pls_create_synthetic(C.byref(spec), options_text(options), C.byref(out)))
        return cls(out)

    @classmethod
    def synthetic_dist(cls, dim, Nel, seed, delta, options: dict, comm):
        """This rank's share of the synthetic system on ``comm`` (lib/dist.py).

        Sizes and vectors are rank-local: [s_r | f_r | p_r] (PETSc row slabs)."""
        spec = N.pls_synth_spec(int(dim), int(Nel), int(seed), float(delta))
        out = C.c_void_p()
        N.check(N.lib().pls_create_synthetic_dist(C.byref(spec), options_text(options), comm.ptr, C.byref(out)))
        h = cls(out)
        h._comm = comm  # destroyed after the handle
        return h

    def update_matrices(self, A=None, P=None, P_diff=None):
        """New values / patterns for the next solves (pls_update_matrices); the
        block PC is set up again before the next solve."""
        keep = []

        def mk(M):
            if M is None:
                return None
            ai, aj, av, nr, nc = N.csr_of(M)
            keep.extend([ai, aj, av])
            return C.byref(N.pls_csr(nr, nc, ai.ctypes.data, aj.ctypes.data, av.ctypes.data))

        N.check(N.lib().pls_update_matrices(self.ptr, mk(A), mk(P), mk(P_diff)))

    # ------------------------------------------------------------- control --
    def set_option(self, key, value=None):
        N.check(N.lib().pls_set_option(self.ptr, str(key).encode(), None if value is None else str(value).encode()))

    def setup(self):
        N.check(N.lib().pls_setup(self.ptr))

    def create_solver(self):
        N.check(N.lib().pls_create_solver(self.ptr))

    def destroy(self):
        if self.ptr:
            N.lib().pls_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    # --------------------------------------------------------- host vectors --
    def pc_apply(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.empty_like(x)
        N.check(N.lib().pls_pc_apply(self.ptr, N.ptr(x), N.ptr(y)))
        return y

    def matmult(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.empty_like(x)
        N.check(N.lib().pls_matmult(self.ptr, N.ptr(x), N.ptr(y)))
        return y

    def solve(self, b):
        b = np.ascontiguousarray(b, dtype=np.float64)
        x = np.empty_like(b)
        r = N.pls_result()
        N.check(N.lib().pls_solve(self.ptr, N.ptr(b), N.ptr(x), C.byref(r)))
        return x, r

    # ------------------------------------------------------- device vectors --
    def solve_device(self, d_b, d_x):
        r = N.pls_result()
        N.check(N.lib().pls_solve_device(self.ptr, d_b, d_x, C.byref(r)))
        return r

    def pc_apply_device(self, d_x, d_y):
        N.check(N.lib().pls_pc_apply_device(self.ptr, d_x, d_y))

    def matmult_device(self, d_x, d_y):
        N.check(N.lib().pls_matmult_device(self.ptr, d_x, d_y))

    def rhs_device(self, seed, d_b):
        N.check(N.lib().pls_synthetic_rhs_device(self.ptr, int(seed), d_b))

    def bench_spmv(self, d_x, d_y, reps):
        s = C.c_double()
        N.check(N.lib().pls_bench_spmv(self.ptr, d_x, d_y, int(reps), C.byref(s)))
        return s.value

    def bench_global_sum(self, count, reps):
        s = C.c_double()
        N.check(N.lib().pls_bench_global_sum(self.ptr, int(count), int(reps), C.byref(s)))
        return s.value

    def spmv_layout(self):
        """(is SELL-64/D16, matrix bytes streamed per product of A)."""
        d, b = C.c_int32(), C.c_int64()
        N.check(N.lib().pls_spmv_layout(self.ptr, C.byref(d), C.byref(b)))
        return bool(d.value), b.value

    # -------------------------------------------------------------- queries --
    def result(self):
        r = N.pls_result()
        N.check(N.lib().pls_get_result(self.ptr, C.byref(r)))
        return r

    def history(self):
        r = self.result()
        h = np.zeros(max(r.history_len, 1), dtype=np.float64)
        N.check(N.lib().pls_get_history(self.ptr, N.ptr(h), r.history_len))
        return h[:r.history_len]

    def timings(self):
        t = N.pls_timings()
        N.check(N.lib().pls_get_timings(self.ptr, C.byref(t)))
        return {f: getattr(t, f) for f, _ in t._fields_}

    def ksp_stats(self, prefix):
        """(solves, iterations, most iterations of one solve, solves with a negative reason,
        the most recent negative reason) of the inner solver with this options prefix
        (pls_get_ksp_stats)."""
        s = np.zeros(5, dtype=np.int64)
        N.check(N.lib().pls_get_ksp_stats(self.ptr, prefix.encode(), N.ptr(s)))
        return tuple(int(v) for v in s)

    def reset_timings(self):
        N.check(N.lib().pls_reset_timings(self.ptr))

    def export_matrix(self, which=0):
        import scipy.sparse as sp
        nr, nnz = C.c_int64(), C.c_int64()
        N.check(N.lib().pls_export_matrix(self.ptr, which, C.byref(nr), C.byref(nnz), None, None, None))
        rp = np.zeros(nr.value + 1, dtype=np.int64)
        ci = np.zeros(nnz.value, dtype=np.int32)
        v = np.zeros(nnz.value, dtype=np.float64)
        N.check(N.lib().pls_export_matrix(self.ptr, which, C.byref(nr), C.byref(nnz), N.ptr(rp), N.ptr(ci), N.ptr(v)))
        return sp.csr_matrix((v, ci, rp), shape=(nr.value, nr.value))

    def permutation(self):
        p = np.zeros(self.n, dtype=np.int64)
        N.check(N.lib().pls_get_permutation(self.ptr, N.ptr(p)))
        return p


def boomeramg_host_level(A, options: dict, prefix: str, level: int):
    """Level ``level`` of the classical AMG hierarchy (-pc_type hypre) that
    libpls builds from ``A`` on the host (``pls_boomeramg_host_level``; no
    device needed): (nlevels, n, nc, cf int8[n], P scipy CSR); on the coarsest
    level cf is empty and P is the coarsest operator."""
    import scipy.sparse as sp
    ai, aj, av, nr, nc_ = N.csr_of(A)
    m = N.pls_csr(nr, nc_, ai.ctypes.data_as(C.c_void_p), aj.ctypes.data_as(C.c_void_p), av.ctypes.data_as(C.c_void_p))
    nl, n, nc, nnz = (C.c_int64() for _ in range(4))
    args = [C.byref(m), options_text(options), prefix.encode(), int(level), C.byref(nl), C.byref(n), C.byref(nc),
            C.byref(nnz)]
    N.check(N.lib().pls_boomeramg_host_level(*args, None, None, None, None))
    cf = np.zeros(n.value if level < nl.value - 1 else 0, dtype=np.int8)
    rp = np.zeros(n.value + 1, dtype=np.int64)
    ci = np.zeros(max(nnz.value, 1), dtype=np.int32)
    v = np.zeros(max(nnz.value, 1), dtype=np.float64)
    N.check(N.lib().pls_boomeramg_host_level(*args, cf.ctypes.data_as(C.c_void_p) if cf.size else None,
                                             rp.ctypes.data_as(C.c_void_p), ci.ctypes.data_as(C.c_void_p),
                                             v.ctypes.data_as(C.c_void_p)))
    ncols = nc.value if level < nl.value - 1 else n.value
    P = sp.csr_matrix((v[:nnz.value], ci[:nnz.value], rp), shape=(n.value, ncols))
    return nl.value, n.value, nc.value, cf, P


LU_STATS = ("n", "fronts", "levels", "max_front", "solve_doubles", "workspace_doubles", "flops", "order_s",
            "symbolic_s", "max_separator")


def sparse_lu_analyze(A, options: dict | None = None, tree: bool = False):
    """Ordering + symbolic analysis of the sparse LU libpls would build on the
    square matrix ``A`` (``pls_sparse_lu_analyze``; host only, no device):
    fronts, tree levels, largest front, doubles one solve reads, doubles
    stored, factorization flops, timings (keys: ``LU_STATS``).  With
    ``tree``: (stats, perm, front_of, parent) -- ND position -> row, position ->
    front (postorder numbers), the fronts' parents."""
    ai, aj, av, nr, nc_ = N.csr_of(A)
    m = N.pls_csr(nr, nc_, ai.ctypes.data_as(C.c_void_p), aj.ctypes.data_as(C.c_void_p), av.ctypes.data_as(C.c_void_p))
    out = (C.c_double * len(LU_STATS))()
    N.check(N.lib().pls_sparse_lu_analyze(C.byref(m), options_text(options or {}), out, len(LU_STATS), None, None,
                                          None))
    stats = dict(zip(LU_STATS, list(out)))
    if not tree:
        return stats
    perm, front_of = np.zeros(nr, dtype=np.int32), np.zeros(nr, dtype=np.int32)
    parent = np.zeros(int(stats["fronts"]), dtype=np.int32)
    N.check(N.lib().pls_sparse_lu_analyze(C.byref(m), options_text(options or {}), out, len(LU_STATS),
                                          perm.ctypes.data_as(C.c_void_p), front_of.ctypes.data_as(C.c_void_p),
                                          parent.ctypes.data_as(C.c_void_p)))
    return stats, perm, front_of, parent
