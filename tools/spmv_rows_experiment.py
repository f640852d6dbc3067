"""Diagnostics: SpMV cost of the pressure rows vs the solid/fluid rows.

Builds the synthetic 3-D system, exports A, and times pls_bench_spmv on
(a) A, (b) A with only the p rows kept (other rows: diagonal only),
(c) A with the p rows reduced to their diagonal.  Prints ns/entry.
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poroelasticity-linear-solvers_amd")]

import lib._native as N  # noqa: E402
from lib.handle import Handle  # noqa: E402


def main(Nel=40):
    N.check(N.lib().pls_set_device(0))
    opts = {"pls.pc_type": "diagonal", "pls.inner_pc_type": "jacobi", "s_pc_type": "jacobi", "fp_pc_type": "jacobi"}
    h = Handle.synthetic(3, Nel, 20261015, 0.05, opts)
    ns, nf, np_ = h.ns, h.nf, h.np
    A = h.export_matrix(0)
    n = A.shape[0]
    print(f"N={Nel} n={n} nnz={A.nnz}", flush=True)
    rows_p = np.zeros(n, dtype=bool)
    rows_p[ns + nf:] = True
    D = sp.diags(A.diagonal()).tocsr()
    Ap = (sp.diags(rows_p.astype(float)) @ A + sp.diags((~rows_p).astype(float)) @ D).tocsr()
    Asf = (sp.diags((~rows_p).astype(float)) @ A + sp.diags(rows_p.astype(float)) @ D).tocsr()
    is_s = np.arange(ns, dtype=np.int32)
    is_f = np.arange(ns, ns + nf, dtype=np.int32)
    is_p = np.arange(ns + nf, n, dtype=np.int32)
    x = N.DeviceArray(n)
    x.upload(np.random.default_rng(0).standard_normal(n))
    y = N.DeviceArray(n)
    for name, M in (("A", A), ("p rows only", Ap), ("s/f rows only", Asf)):
        hh = Handle.from_csr(M, M, None, is_s, is_f, is_p, [], opts)
        hh.bench_spmv(x.p, y.p, 3)
        t = hh.bench_spmv(x.p, y.p, 20)
        d16, mb = hh.spmv_layout()
        print(f"{name:14s} nnz {M.nnz:11d}  {t * 1e3:8.3f} ms  {t / M.nnz * 1e12:7.2f} ps/entry  "
              f"layout {mb / t / 1e9:7.1f} GB/s  d16={d16}", flush=True)
        hh.destroy()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 40)
