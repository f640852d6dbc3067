"""Diagnostics: device SpMV (outer-operator path) on odd CSR shapes vs scipy."""
import sys
sys.path[:0] = ["/root/repo", "/root/repo/tests", "/root/repo/poroelasticity-linear-solvers_amd"]
import numpy as np
import scipy.sparse as sp
from oracle import synthetic as S
import test_gpu_amg as T
from test_gpu_parity import BASE, _oracle
from lib.handle import Handle


def check(name, M, opts=None):
    n = M.shape[0]
    M = sp.csr_matrix(M)
    M.sort_indices()
    k = n // 3
    iss, isf, isp = np.arange(0, k), np.arange(k, 2 * k), np.arange(2 * k, n)
    I = sp.eye(n, format="csr")
    h = Handle.from_csr(M, I, I, iss, isf, isp, None, dict({"pls.pc_type": "diagonal"}, **(opts or {})))
    x = np.random.default_rng(0).standard_normal(n)
    y = h.matmult(x)
    ref = M @ x
    sc = abs(M) @ np.abs(x) + 1e-300
    print(name, "n", n, "nnz", M.nnz, "maxrow", np.diff(M.indptr).max(), "layout", h.spmv_layout(),
          "rel err", np.max(np.abs(y - ref) / sc), flush=True)


spec = S.SynthSpec(3, 5)
params = dict(BASE, **{"pc type": "diagonal 3-way", "inner pc type": "lu"})
o = _oracle(spec, params, T._amg_db("gamg"))
L = o.block_pc.ksp_s.pc.levels[0]
A, P, R = L["A"], L["P"], L["R"]
n = A.shape[0]
Rsq = sp.vstack([R, sp.csr_matrix((n - R.shape[0], n))]).tocsr() + sp.diags(np.r_[np.zeros(R.shape[0]), np.ones(n - R.shape[0])])
Psq = sp.hstack([P, sp.csr_matrix((n, n - P.shape[1]))]).tocsr()
check("A_s", A)
check("R_s(square)", Rsq)
check("P_s(square)", Psq)
check("R_s(square) nod16", Rsq, {"pls.sell_d16": "0"})
for rows in (1, 5, 14, 63, 64, 65, 130):
    rng = np.random.default_rng(rows)
    m = 4000
    B = sp.random(rows, m, density=0.7, random_state=rows, format="csr")
    Bsq = (sp.vstack([B, sp.csr_matrix((m - rows, m))]) + sp.eye(m)).tocsr()
    check(f"long rows x{rows}", Bsq)
