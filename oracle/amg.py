"""Smoothed-aggregation AMG preconditioner (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

The reference's inexact option set solves its s_ / f_ / p_ / diff_ /
fp_fieldsplit_0_ blocks with CG + hypre BoomerAMG (``petsc-options-inexact``,
SURVEY.md 8(f) rank 3).  hypre is absent from this image and from the
reference tree, so its numerics cannot be restated or pinned.  libpls
provides a GPU algebraic multigrid instead -- PETSc-GAMG-like smoothed
aggregation -- used for ``-pc_type gamg`` and, unless ``pls.hypre error`` is
set, as the stand-in for ``-pc_type hypre``.  This module is the exact
specification the device implementation (csrc/amg.cpp) follows and the
oracle the GPU tests compare it with.  Iteration counts differ from
BoomerAMG's; parity is against this spec.

Setup, level l (A_l square, CSR, sorted):
* strength: W = |A| + |A|^T off the diagonal; j is a strong neighbour of i iff
  W_ij > 2 theta sqrt(|a_ii a_jj|)   (theta = -pc_gamg_threshold, default 0);
* aggregation, deterministic:
  pass 1: rows in order; an unaggregated row whose strong neighbours are all
          unaggregated starts an aggregate with them;
  pass 2: every row left joins the pass-1 aggregate of its neighbour with the
          largest W_ij (ties: smallest j);
  pass 3: rows still left are singletons;
  stop when no coarsening happens;
* tentative prolongator P0[i, agg(i)] = 1 / sqrt(|agg(i)|);
* lambda = power iteration on D^-1 A, 15 steps from v = 1:
  w = D^-1 A v, lambda = ||w|| / ||v||, v = w / ||w||; lambda is rounded to
  float32 so the hierarchy does not hinge on the norms' summation order;
* P = P0 - (4 / (3 lambda)) D^-1 A P0;   R = P^T;   A_{l+1} = R (A P);
* levels stop at n <= -pc_gamg_coarse_eq_limit (50) or -pc_mg_levels (10);
  the coarsest level is solved exactly (LU).
V-cycle (one PC application y = M^-1 b): x = 0; K = -mg_levels_ksp_max_it (2;
for the hypre stand-in -pc_hypre_boomeramg_grid_sweeps_all, default 1)
Chebyshev steps with Jacobi on [0.1 lambda, 1.1 lambda] (Saad, Alg. 12.1:
theta = (max+min)/2, delta = (max-min)/2, sigma = theta/delta, rho = 1/sigma,
r = b - A x, d = D^-1 r / theta, then K times: x += d, and unless last:
r = b - A x, rho' = 1/(2 sigma - rho), d = rho' rho d + (2 rho'/delta) D^-1 r);
r = b - A x; recurse on R r; x += P e; K Chebyshev steps again.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from .options import get as opt


def aggregate(A, theta=0.0):
    A = A.tocsr()
    n = A.shape[0]
    d = np.abs(A.diagonal())
    absA = abs(A)
    W = (absA + absA.T).tocsr()
    W.setdiag(0.0)
    W.eliminate_zeros()
    W.sort_indices()
    rp, ci, wv = W.indptr, W.indices, W.data
    strong_lists = []
    for i in range(n):
        js = ci[rp[i]:rp[i + 1]]
        ws = wv[rp[i]:rp[i + 1]]
        keep = ws > 2.0 * theta * np.sqrt(d[i] * d[js])
        strong_lists.append((js[keep], ws[keep]))
    agg = -np.ones(n, dtype=np.int64)
    na = 0
    for i in range(n):
        js, _ = strong_lists[i]
        if agg[i] < 0 and np.all(agg[js] < 0):
            agg[i] = na
            agg[js] = na
            na += 1
    agg1 = agg.copy()
    for i in range(n):
        if agg1[i] >= 0:
            continue
        js, ws = strong_lists[i]
        best, bestw = -1, -1.0
        for j, w in zip(js, ws):
            if agg1[j] >= 0 and w > bestw:
                best, bestw = j, w
        if best >= 0:
            agg[i] = agg1[best]
    for i in range(n):
        if agg[i] < 0:
            agg[i] = na
            na += 1
    return agg, na


def power_lambda(A, dinv, steps=15):
    v = np.ones(A.shape[0])
    lam = 1.0
    for _ in range(steps):
        w = dinv * (A @ v)
        nw, nv = np.linalg.norm(w), np.linalg.norm(v)
        if nw == 0.0:
            return 1.0
        lam = nw / nv
        v = w / nw
    return lam


def _dinv(A):
    d = A.diagonal().astype(np.float64)
    return np.where(d != 0.0, 1.0 / np.where(d != 0.0, d, 1.0), 1.0)


class PCAMG:
    type = "gamg"

    def __init__(self, A, db=None, prefix="", hypre=False):
        db = db or {}
        theta = opt(db, prefix, "pc_gamg_threshold", 0.0, float)
        limit = opt(db, prefix, "pc_gamg_coarse_eq_limit", 50, int)
        maxlev = opt(db, prefix, "pc_mg_levels", 10, int)
        ksweeps = opt(db, prefix, "pc_hypre_boomeramg_grid_sweeps_all", 1, int) if hypre else 2
        self.K = opt(db, prefix, "mg_levels_ksp_max_it", ksweeps, int)
        if self.K < 1:
            raise ValueError("mg_levels_ksp_max_it must be >= 1")
        A = A.tocsr()
        A.sort_indices()
        self.levels = []
        while A.shape[0] > limit and len(self.levels) < maxlev - 1:
            agg, na = aggregate(A, theta)
            if na >= A.shape[0] or na == 0:
                break
            n = A.shape[0]
            sizes = np.bincount(agg, minlength=na).astype(np.float64)
            P0 = sp.csr_matrix((1.0 / np.sqrt(sizes[agg]), (np.arange(n), agg)), shape=(n, na))
            dinv = _dinv(A)
            lam = float(np.float32(power_lambda(A, dinv)))
            P = (P0 - (4.0 / (3.0 * lam)) * (sp.diags(dinv) @ (A @ P0))).tocsr()
            P.sort_indices()
            R = P.T.tocsr()
            R.sort_indices()
            Ac = (R @ (A @ P)).tocsr()
            Ac.sort_indices()
            self.levels.append({"A": A, "dinv": dinv, "lam": lam, "P": P, "R": R})
            A = Ac
        self.coarse = A
        self.coarse_lu = spla.splu(sp.csc_matrix(A))

    def _cheb(self, L, b, x):
        A, dinv, lam = L["A"], L["dinv"], L["lam"]
        lmax, lmin = 1.1 * lam, 0.1 * lam
        theta, delta = (lmax + lmin) / 2.0, (lmax - lmin) / 2.0
        sigma = theta / delta
        rho = 1.0 / sigma
        r = b - A @ x
        d = (dinv * r) * (1.0 / theta)
        for k in range(self.K):
            x = x + d
            if k == self.K - 1:
                break
            r = b - A @ x
            rho_n = 1.0 / (2.0 * sigma - rho)
            d = (rho_n * rho) * d + (2.0 * rho_n / delta) * (dinv * r)
            rho = rho_n
        return x

    def _vcycle(self, l, b):
        if l == len(self.levels):
            return self.coarse_lu.solve(b)
        L = self.levels[l]
        x = self._cheb(L, b, np.zeros_like(b))
        r = b - L["A"] @ x
        e = self._vcycle(l + 1, L["R"] @ r)
        x = x + L["P"] @ e
        return self._cheb(L, b, x)

    def apply(self, b):
        b = np.asarray(b, dtype=np.float64)
        if b.size == 0:
            return b.copy()
        return self._vcycle(0, b)
