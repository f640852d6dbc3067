"""AAR and inner Anderson acceleration restated (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Single-process transcription of
* reference ``lib/AAR.py:46-137`` (``AAR.solve`` / ``update_residual``), and
* reference ``lib/AndersonAcceleration.py:19-78`` (``get_next_vector``),
keeping every quirk the survey lists:
  - f_0 is the UNpreconditioned residual b - A x0 (AAR.py:55-56) and seeds the
    first difference Delta f_0 = M^-1 r_0 - r_0 (AAR.py:75-78);
  - Richardson unless it > 0, order > 0 and (it + 1) % p == 0 (AAR.py:94);
  - the Anderson least squares uses every stored F column (it + 1 of them
    during warm-up) but only the first mk = min(order, it) coefficients are
    applied, paired with X[i] and F[i] (AAR.py:99-111);
  - numpy Householder QR then ``solve(R, -Q^T f)`` (AAR.py:102-105);
  - stop test on ||M^-1 r_k|| / ||b - A x0|| (AAR.py:117-118);
  - the F / X histories persist across ``solve`` calls (AAR.py:20-22).
"""
from __future__ import annotations

import numpy as np


def _householder_r(A):
    """R (m x m, upper) of a rows x m panel by the reflections libpls's k_tsqr
    applies (LAPACK dlarfg conventions)."""
    A = np.array(A, dtype=np.float64)
    rows, m = A.shape
    for j in range(min(m, rows)):
        sigma = float(A[j + 1:, j] @ A[j + 1:, j])
        alpha = A[j, j]
        if sigma == 0.0:
            continue
        nrm = np.sqrt(alpha * alpha + sigma)
        beta = -nrm if alpha >= 0.0 else nrm
        tau, scal = (beta - alpha) / beta, 1.0 / (alpha - beta)
        for k in range(j + 1, m):
            w = A[j, k] + scal * float(A[j + 1:, j] @ A[j + 1:, k])
            A[j, k] -= tau * w
            A[j + 1:, k] -= tau * w * (A[j + 1:, j] * scal)
        A[j, j] = beta
    out = np.zeros((m, m))
    k = min(m, rows)
    out[:k] = np.triu(A[:k])
    return out


def tsqr_lstsq(F, f, rows_per_block=512):
    """min ||f + F a|| the way libpls solves it (csrc/capi.cpp AndersonLS):
    Householder TSQR of [F | f] over 512-row chunks, then of the stacked R's
    until one is left; a = R^-1 (-z) with z the last column.  Used by the tests
    to measure how far two backward-stable solvers of the same least squares
    drift apart in a whole AAR history (the noise floor of the comparison)."""
    P = np.column_stack([F, f])
    m = P.shape[1]
    while True:
        n = P.shape[0]
        nch = -(-n // rows_per_block)
        P = np.vstack([_householder_r(P[b * rows_per_block:(b + 1) * rows_per_block]) for b in range(nch)])
        if nch == 1:
            break
    L = m - 1
    return np.linalg.solve(P[:L, :L], -P[:L, L])


class AAR:
    def __init__(self, order, p, omega, beta, A, pc, atol=1e-12, rtol=1e-8, maxiter=1000,
                 monitor=None):
        self.order, self.p, self.omega, self.beta = order, p, omega, beta
        self.A, self.pc = A, pc
        self.atol, self.rtol, self.maxiter = atol, rtol, maxiter
        self.monitor = monitor
        self.F, self.X, self.F0 = [], [], []
        self.it = 0
        self.history = []
        self.max_cond = 1.0  # largest cond(F) met in an Anderson least squares
        self.lstsq = None  # tests only: another backward-stable solver of min ||f + F a|| (noise floor)

    def _update_residual(self, b, xk):
        temp = b - self.A @ xk
        return self.pc.apply(temp)

    def solve(self, b):
        b = np.asarray(b, dtype=np.float64)
        x0 = np.zeros_like(b)
        xk = x0.copy()
        fk = b - self.A @ x0
        error0 = float(np.linalg.norm(fk))
        err_abs, err_rel, it = error0, 1.0, 0
        self.history = [error0]
        while err_abs > self.atol and err_rel > self.rtol and it < self.maxiter:
            delta_fk = fk.copy()
            delta_xk = xk.copy()
            fk = self._update_residual(b, xk)
            delta_fk = fk - delta_fk
            self.F.append(delta_fk.copy())
            if len(self.F) > self.order:
                self.F.pop(0)
            self.F0.append(delta_fk.copy())
            if len(self.F0) > self.order:
                self.F0.pop(0)
            if float(np.linalg.norm(fk)) < 1e-14:
                pass
            elif it == 0 or self.order == 0 or (it + 1) / self.p % 1 > 0:
                xk = xk + self.omega * fk
            else:
                mk = min(self.order, it)
                F = np.vstack(self.F0).T
                Q, R = np.linalg.qr(F)
                alpha = np.linalg.solve(R, -Q.T @ fk) if self.lstsq is None else self.lstsq(F, fk)
                self.max_cond = max(self.max_cond, float(np.linalg.cond(R)))
                xk = xk + self.beta * fk
                for i in range(mk):
                    xk = xk + alpha[i] * (self.X[i] + self.beta * self.F[i])
            delta_xk = xk - delta_xk
            self.X.append(delta_xk.copy())
            if len(self.X) > self.order:
                self.X.pop(0)
            err_abs = float(np.linalg.norm(fk))
            err_rel = err_abs / error0
            it += 1
            self.history.append(err_abs)
            if self.monitor:
                self.monitor(it, err_abs, err_rel)
        self.it = it
        return xk

    def getIterationNumber(self):
        return self.it


class AndersonAcceleration:
    def __init__(self, order):
        self.order = order
        self.k = 0
        self.F, self.X, self.F0 = [], [], []
        self.max_cond = 1.0
        self.lstsq = None

    def get_next_vector(self, gk):
        gk = np.asarray(gk, dtype=np.float64)
        if self.k == 0:
            self.xk = np.zeros_like(gk)
            self.fk = np.zeros_like(gk)
        delta_fk = self.fk.copy()
        delta_xk = self.xk.copy()
        self.fk = gk - self.xk
        mk = min(self.k, self.order)
        if mk > 0:
            delta_fk = self.fk - delta_fk
            if float(np.linalg.norm(delta_fk)) < 1e-12:
                self.k -= 1
                self.xk = gk.copy()
            else:
                self.F.append(delta_fk.copy())
                if len(self.F) > self.order:
                    self.F.pop(0)
                self.F0.append(delta_fk.copy())
                if len(self.F0) > self.order:
                    self.F0.pop(0)
                F = np.vstack(self.F0).T
                Q, R = np.linalg.qr(F)
                alpha = np.linalg.solve(R, -Q.T @ self.fk) if self.lstsq is None else self.lstsq(F, self.fk)
                self.max_cond = max(self.max_cond, float(np.linalg.cond(R)))
                self.xk = self.xk + 1.0 * self.fk
                for i in range(mk):
                    self.xk = self.xk + alpha[i] * (self.X[i] + self.F[i])
        else:
            self.xk = gk.copy()
        delta_xk = self.xk - delta_xk
        self.X.append(delta_xk.copy())
        if len(self.X) > self.order:
            self.X.pop(0)
        self.k += 1
        return self.xk.copy()
