"""PETSc KSP / PC semantics as the reference configures them (TEST INFRASTRUCTURE ONLY).

PETSc is a third-party dependency absent from /root/reference (version
unpinned; see oracle/__init__.py).  Restated from PETSc's published algorithms:

* ``KSPConvergedDefault`` (iterativ.c): at n == 0 with a zero initial guess
  rnorm0 = rnorm, ttol = max(rtol * rnorm0, atol); converged when
  rnorm <= ttol (ATOL if rnorm < atol else RTOL); NaN/Inf -> DIVERGED_NANORINF;
  rnorm >= dtol * rnorm0 -> DIVERGED_DTOL.
* ``KSPGMRES`` (gmres.c): restarted GMRES, classical Gram-Schmidt without
  refinement (VecMDot then VecMAXPY with -h), VecScale by 1/||w||, happy
  breakdown when ||w|| < min(|||w|| / g_k|, haptol=1e-30), Givens rotations
  (KSPGMRESUpdateHessenberg), back substitution and, for right
  preconditioning, one more PC apply in BuildSoln (KSPUnwindPreconditioner).
  Left PC: Krylov operator B A, preconditioned norm.  Right PC: A B,
  unpreconditioned norm.  The reference configures the outer solver at
  ``lib/Solver.py:91-102`` (restart = maxit, dtol = 1e20, zero guess).
* ``KSPCG`` (cg.c) with PRECONDITIONED / UNPRECONDITIONED norms.
* ``KSPPREONLY``: x = B b, its = 1, CONVERGED_ITS.
* PCs NONE, JACOBI (multiply by 1/diag; zero diag -> 1), ILU (ILU(0), natural
  ordering; oracle/csrc/oracle.c), BJACOBI (PETSc block sizing: the first
  n % nblocks blocks get one extra row; sub-KSP PREONLY, sub-PC ILU(0)), and
  LU (scipy splu: the exact solve MUMPS provides in the reference's
  ``petsc-options-exact``).
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from . import native
from .options import get as opt

# KSPConvergedReason values (petscksp.h)
CONVERGED_RTOL = 2
CONVERGED_ATOL = 3
CONVERGED_ITS = 4
CONVERGED_HAPPY_BREAKDOWN = 5
CONVERGED_ITERATING = 0
DIVERGED_NULL = -2
DIVERGED_ITS = -3
DIVERGED_DTOL = -4
DIVERGED_BREAKDOWN = -5
DIVERGED_INDEFINITE_PC = -8
DIVERGED_NANORINF = -9
DIVERGED_INDEFINITE_MAT = -10

PETSC_DEFAULT_RTOL = 1e-5
PETSC_DEFAULT_ATOL = 1e-50
PETSC_DEFAULT_DTOL = 1e4
PETSC_DEFAULT_MAXIT = 10000
GMRES_DEFAULT_RESTART = 30
GMRES_HAPTOL = 1e-30


# ------------------------------------------------------------------- PCs ----
class PCNone:
    type = "none"

    def apply(self, x):
        return np.array(x, dtype=np.float64, copy=True)


class PCJacobi:
    type = "jacobi"

    def __init__(self, M):
        d = M.diagonal().astype(np.float64)
        d[d == 0.0] = 1.0
        self.dinv = 1.0 / d

    def apply(self, x):
        return x * self.dinv


class PCILU:
    type = "ilu"

    def __init__(self, M, levels: int = 0):
        if levels != 0:
            raise NotImplementedError("only ILU(0) is restated")
        self.f = native.ILU0(M)

    def apply(self, x):
        return self.f.solve(x)


class PCLU:
    type = "lu"

    def __init__(self, M):
        self.f = spla.splu(sp.csc_matrix(M))

    def apply(self, x):
        return self.f.solve(np.asarray(x, dtype=np.float64))


def bjacobi_block_sizes(n: int, nblocks: int):
    """PCBJACOBI default split (bjacobi.c): l_lens[i] = n/B + ((n % B) > i)."""
    return [n // nblocks + (1 if (n % nblocks) > i else 0) for i in range(nblocks)]


class PCBJacobi:
    type = "bjacobi"

    def __init__(self, M, nblocks: int = 1, sub_pc_type: str = "ilu"):
        M = M.tocsr()
        n = M.shape[0]
        nblocks = max(1, min(int(nblocks), n))
        lens = bjacobi_block_sizes(n, nblocks)
        self.bounds = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        self.subs = []
        for b in range(nblocks):
            lo, hi = self.bounds[b], self.bounds[b + 1]
            self.subs.append(make_pc_of_type(sub_pc_type, M[lo:hi, lo:hi].tocsr()))

    def apply(self, x):
        y = np.empty_like(x)
        for b, s in enumerate(self.subs):
            lo, hi = self.bounds[b], self.bounds[b + 1]
            y[lo:hi] = s.apply(x[lo:hi])
        return y


class PCShell:
    type = "python"

    def __init__(self, fn):
        self.fn = fn

    def apply(self, x):
        return self.fn(x)


def make_pc_of_type(t, M, db=None, prefix=""):
    db = db or {}
    if t in ("none",):
        return PCNone()
    if t == "jacobi":
        return PCJacobi(M)
    if t == "ilu":
        return PCILU(M, opt(db, prefix, "pc_factor_levels", 0, int))
    if t == "lu" or t == "cholesky":
        return PCLU(M)
    if t == "bjacobi":
        return PCBJacobi(M, opt(db, prefix, "pc_bjacobi_blocks", 1, int),
                         opt(db, prefix + "sub_", "pc_type", "ilu"))
    if t == "hypre":
        h = str(db.get("pls.hypre", "boomeramg"))
        if h == "error":
            raise NotImplementedError("PC type 'hypre' is not available (pls.hypre error)")
        if h in ("sa", "gamg"):
            from .amg import PCAMG
            return PCAMG(M, db, prefix, hypre=True)
        from .boomeramg import PCBoomerAMG
        return PCBoomerAMG(M, db, prefix)
    if t == "gamg":
        from .amg import PCAMG
        return PCAMG(M, db, prefix)
    raise NotImplementedError(f"PC type '{t}' is not restated by the oracle")


# ---------------------------------------------------------- convergence ----
class ConvergedDefault:
    def __init__(self, rtol, atol, dtol):
        self.rtol, self.atol, self.dtol = rtol, atol, dtol
        self.rnorm0 = None
        self.ttol = None

    def __call__(self, n, rnorm):
        if n == 0:
            self.rnorm0 = rnorm
            self.ttol = max(self.rtol * self.rnorm0, self.atol)
        if math.isnan(rnorm) or math.isinf(rnorm):
            return DIVERGED_NANORINF
        if rnorm <= self.ttol:
            return CONVERGED_ATOL if rnorm < self.atol else CONVERGED_RTOL
        if rnorm >= self.dtol * self.rnorm0:
            return DIVERGED_DTOL
        return CONVERGED_ITERATING


# ------------------------------------------------------------------ KSPs ----
class KSP:
    """A configured KSP (type, tolerances, side, norm, PC) on operator A."""

    def __init__(self, A, pc, ksp_type="gmres", rtol=PETSC_DEFAULT_RTOL,
                 atol=PETSC_DEFAULT_ATOL, dtol=PETSC_DEFAULT_DTOL,
                 maxit=PETSC_DEFAULT_MAXIT, restart=GMRES_DEFAULT_RESTART,
                 pc_side=None, norm_type=None, monitor=None):
        self.A, self.pc, self.type = A, pc, ksp_type
        self.rtol, self.atol, self.dtol, self.maxit = rtol, atol, dtol, int(maxit)
        self.restart = int(restart)
        self.pc_side, self.norm_type = resolve_side_norm(ksp_type, pc_side, norm_type)
        self.its = 0
        self.reason = 0
        self.history = []
        self.monitor = monitor

    def matvec(self, x):
        return self.A @ x

    # inner products (oracle/dist.py overrides them with rank-ordered global sums)
    def dot(self, a, b):
        return float(np.dot(a, b))

    def norm(self, a):
        return float(np.linalg.norm(a))

    def solve(self, b):
        b = np.asarray(b, dtype=np.float64)
        if self.type == "preonly":
            x = self.pc.apply(b)
            self.its, self.reason, self.history = 1, CONVERGED_ITS, []
            return x
        if self.type == "gmres":
            return _gmres(self, b)
        if self.type == "cg":
            return _cg(self, b)
        raise NotImplementedError(f"KSP type '{self.type}' is not restated by the oracle")


def resolve_side_norm(ksp_type, pc_side, norm_type):
    """KSPSetUpNorms_Private: pick the (norm, side) pair the type supports.

    GMRES: (preconditioned, left) default; unpreconditioned => right.
    CG: left only; preconditioned default.  PREONLY: norm none.
    """
    if ksp_type == "preonly":
        return "left", "none"
    if ksp_type == "gmres":
        if pc_side is None:
            pc_side = "right" if norm_type == "unpreconditioned" else "left"
        if norm_type is None:
            norm_type = "unpreconditioned" if pc_side == "right" else "preconditioned"
        if (pc_side, norm_type) not in (("left", "preconditioned"), ("right", "unpreconditioned"),
                                        ("left", "none"), ("right", "none")):
            raise ValueError(f"GMRES does not support norm {norm_type} with pc side {pc_side}")
        return pc_side, norm_type
    if ksp_type == "cg":
        if pc_side not in (None, "left"):
            raise ValueError(f"{ksp_type} supports only left preconditioning")
        return "left", (norm_type or "preconditioned")
    return pc_side or "left", norm_type or "preconditioned"


def _gmres(ksp: KSP, b):
    """KSPSolve_GMRES + KSPGMRESCycle + KSPGMRESBuildSoln (gmres.c)."""
    n = b.size
    x = np.zeros(n)
    conv = ConvergedDefault(ksp.rtol, ksp.atol, ksp.dtol)
    right = ksp.pc_side == "right"
    max_k = ksp.restart
    its = 0
    reason = 0
    hist = []
    first = True
    while not reason:
        # KSPInitialResidual
        if first:
            r = b.copy()
        else:
            r = b - ksp.matvec(x)
        if not right:
            r = ksp.pc.apply(r)
        # --- cycle
        res = ksp.norm(r)
        V = [r * (1.0 / res) if res != 0.0 else r]
        hist.append(res)
        if ksp.monitor:
            ksp.monitor(its, res)
        if res == 0.0:
            reason = CONVERGED_ATOL
            break
        reason = conv(its, res)
        HH = np.zeros((max_k + 1, max_k + 1))
        cc = np.zeros(max_k + 1)
        ss = np.zeros(max_k + 1)
        grs = np.zeros(max_k + 2)
        grs[0] = res
        loc_it = 0
        while not reason and loc_it < max_k and its < ksp.maxit:
            v = V[loc_it]
            if right:
                w = ksp.matvec(ksp.pc.apply(v))
            else:
                w = ksp.pc.apply(ksp.matvec(v))
            # classical Gram-Schmidt: h = V^T w ; w -= V h
            h = np.array([ksp.dot(V[j], w) for j in range(loc_it + 1)])
            for j in range(loc_it + 1):
                w = w - h[j] * V[j]
            HH[:loc_it + 1, loc_it] = h
            tt = ksp.norm(w)
            HH[loc_it + 1, loc_it] = tt
            hapbnd = abs(tt / grs[loc_it])
            if hapbnd > GMRES_HAPTOL:
                hapbnd = GMRES_HAPTOL
            hapend = tt < hapbnd
            if not hapend:
                with np.errstate(divide="ignore"):
                    inv = np.float64(1.0) / np.float64(tt)  # C semantics: 1/0 = inf (never reused)
                with np.errstate(invalid="ignore", over="ignore"):
                    w = w * inv
            V.append(w)
            # KSPGMRESUpdateHessenberg
            it = loc_it
            for j in range(it):
                t0 = HH[j, it]
                HH[j, it] = cc[j] * t0 + ss[j] * HH[j + 1, it]
                HH[j + 1, it] = cc[j] * HH[j + 1, it] - ss[j] * t0
            if not hapend:
                t0 = math.sqrt(HH[it, it] * HH[it, it] + HH[it + 1, it] * HH[it + 1, it])
                if t0 == 0.0:
                    reason = DIVERGED_NULL
                    break
                cc[it] = HH[it, it] / t0
                ss[it] = HH[it + 1, it] / t0
                grs[it + 1] = -(ss[it] * grs[it])
                grs[it] = cc[it] * grs[it]
                HH[it, it] = cc[it] * HH[it, it] + ss[it] * HH[it + 1, it]
                res = abs(grs[it + 1])
            else:
                res = 0.0
            loc_it += 1
            its += 1
            hist.append(res)
            if ksp.monitor:
                ksp.monitor(its, res)
            reason = conv(its, res)
            if hapend:
                if not reason:
                    reason = DIVERGED_BREAKDOWN
                    break
        # KSPGMRESBuildSoln
        it = loc_it - 1
        if it >= 0:
            if HH[it, it] == 0.0:
                reason = DIVERGED_BREAKDOWN
            else:
                nrs = np.zeros(it + 1)
                nrs[it] = grs[it] / HH[it, it]
                for k in range(it - 1, -1, -1):
                    t0 = grs[k]
                    for j in range(k + 1, it + 1):
                        t0 = t0 - HH[k, j] * nrs[j]
                    nrs[k] = t0 / HH[k, k]
                tmp = np.zeros(n)
                for j in range(it + 1):
                    tmp = tmp + nrs[j] * V[j]
                if right:
                    tmp = ksp.pc.apply(tmp)
                x = x + tmp
        if its >= ksp.maxit:
            if not reason:
                reason = DIVERGED_ITS
            break
        first = False
    ksp.its, ksp.reason, ksp.history = its, reason, hist
    return x


def _cg(ksp: KSP, b):
    """KSPSolve_CG (cg.c), zero initial guess, no eigenvalue estimates."""
    conv = ConvergedDefault(ksp.rtol, ksp.atol, ksp.dtol)
    x = np.zeros_like(b)
    r = b.copy()
    hist = []
    z = None
    if ksp.norm_type == "preconditioned":
        z = ksp.pc.apply(r)
        dp = ksp.norm(z)
    elif ksp.norm_type == "unpreconditioned":
        dp = ksp.norm(r)
    else:
        dp = 0.0
    hist.append(dp)
    if ksp.monitor:
        ksp.monitor(0, dp)
    reason = conv(0, dp) if ksp.norm_type != "none" else 0
    its = 0
    if reason:
        ksp.its, ksp.reason, ksp.history = its, reason, hist
        return x
    if ksp.norm_type != "preconditioned":
        z = ksp.pc.apply(r)
    beta = ksp.dot(z, r)
    i = 0
    p = None
    dpi = 0.0
    betaold = 0.0
    while True:
        its = i + 1
        if beta == 0.0:
            reason = CONVERGED_ATOL
            break
        if i > 0 and beta * betaold < 0.0:  # cg.c: indefinite preconditioner
            reason = DIVERGED_INDEFINITE_PC
            break
        if i == 0:
            p = z.copy()
        else:
            bb = beta / betaold
            p = bb * p + z
        dpiold = dpi
        w = ksp.matvec(p)
        dpi = ksp.dot(p, w)
        betaold = beta
        if dpi == 0.0 or (i > 0 and np.sign(dpi) * np.sign(dpiold) < 0.0):
            reason = DIVERGED_INDEFINITE_MAT
            break
        a = beta / dpi
        x = x + a * p
        r = r + (-a) * w
        if ksp.norm_type == "preconditioned":
            z = ksp.pc.apply(r)
            dp = ksp.norm(z)
        elif ksp.norm_type == "unpreconditioned":
            dp = ksp.norm(r)
        else:
            dp = 0.0
        hist.append(dp)
        if ksp.monitor:
            ksp.monitor(i + 1, dp)
        if ksp.norm_type != "none":
            reason = conv(i + 1, dp)
        if reason:
            break
        if ksp.norm_type != "preconditioned":
            z = ksp.pc.apply(r)
        beta = ksp.dot(z, r)
        i += 1
        if i >= ksp.maxit:
            break
    if i >= ksp.maxit and not reason:
        reason = DIVERGED_ITS
    ksp.its, ksp.reason, ksp.history = its, reason, hist
    return x


# ----------------------------------------------- options -> configured KSP --
def ksp_from_options(prefix, db, A, P, default_ksp_type, default_pc_type,
                     rtol=PETSC_DEFAULT_RTOL, atol=PETSC_DEFAULT_ATOL,
                     dtol=PETSC_DEFAULT_DTOL, maxit=PETSC_DEFAULT_MAXIT,
                     restart=GMRES_DEFAULT_RESTART, pc=None):
    """setType/setTolerances then setFromOptions: the options DB wins."""
    ktype = opt(db, prefix, "ksp_type", default_ksp_type)
    rtol = opt(db, prefix, "ksp_rtol", rtol, float)
    atol = opt(db, prefix, "ksp_atol", atol, float)
    dtol = opt(db, prefix, "ksp_divtol", dtol, float)
    maxit = opt(db, prefix, "ksp_max_it", maxit, int)
    restart = opt(db, prefix, "ksp_gmres_restart", restart, int)
    side = opt(db, prefix, "ksp_pc_side", None)
    norm = opt(db, prefix, "ksp_norm_type", None)
    if pc is None:
        ptype = opt(db, prefix, "pc_type", default_pc_type)
        pc = make_pc_of_type(ptype, P, db, prefix)
    return KSP(A, pc, ktype, rtol, atol, dtol, maxit, restart, side, norm)
