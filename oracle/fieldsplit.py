"""PCFIELDSPLIT as the reference configures it (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

The reference's 2-way preconditioner solves the fluid-pressure block with
GMRES + PCFIELDSPLIT unless the inner PC type is ``lu``
(``lib/Preconditioner.py:102-118``, ``setup_fieldsplit``): splits are set with
``setFieldSplitIS((None, is_p))`` then ``((None, is_f))`` -- split 0 is the
pressure, split 1 the fluid, both in fp-local numbering
(``lib/IndexSet.py:46-54``) -- and ``petsc-options-inexact:73-114`` selects
``schur`` / ``lower`` / ``selfp`` with ``fieldsplit_0`` = CG and
``fieldsplit_1`` = PREONLY + LU.

PETSc (third-party, absent from /root/reference) semantics restated from its
published algorithm (src/ksp/pc/impls/fieldsplit/fieldsplit.c):

* A = [[A00, A01], [A10, A11]] with rows/columns of split i in IS order.
* type (``-pc_fieldsplit_type``, default MULTIPLICATIVE):
  - ADDITIVE: y_i = K_i^-1 x_i;
  - MULTIPLICATIVE: y_0 = K_0^-1 x_0; y_1 = K_1^-1 (x_1 - A10 y_0);
  - SCHUR with ``-pc_fieldsplit_schur_fact_type`` (default FULL):
    DIAG:  y_0 = A00^-1 x_0;  y_1 = s * S^-1 x_1 (s = schur_scale, default -1)
    LOWER: y_0 = A00^-1 x_0;  y_1 = S^-1 (x_1 - A10 y_0)
    UPPER: y_1 = S^-1 x_1;    y_0 = A00^-1 (x_0 - A01 y_1)
    FULL:  t = A00^-1 x_0;  y_1 = S^-1 (x_1 - A10 t);  y_0 = A00^-1 (x_0 - A01 y_1)
* The Schur KSP (prefix ``fieldsplit_1_``, default GMRES) has operator
  S = A11 - A10 A00^-1 A01 (MatSchurComplement, inner solve = the split-0 KSP)
  and preconditioning matrix ``-pc_fieldsplit_schur_precondition``
  (default A11): SELFP = A11 - A10 diag(A00)^-1 A01 (MatSchurComplementGetPmat:
  diag reciprocal with zeros kept 0, row-scaled A01, MatMatMult with the
  product summed over k ascending, then D - S), or A11.
* Split KSPs default to PREONLY (split 0 and non-Schur splits), PC default
  ILU for a sequential AIJ matrix.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

from . import petsc
from .options import get as opt


def selfp(A00, A01, A10, A11):
    """A11 - A10 diag(A00)^-1 A01 (MAT_SCHUR_COMPLEMENT_AINV_DIAG)."""
    d = A00.diagonal().astype(np.float64)
    with np.errstate(divide="ignore"):
        dinv = np.where(d != 0.0, 1.0 / np.where(d != 0.0, d, 1.0), 0.0)
    AinvB = sp.diags(dinv) @ A01.tocsr()
    S = (A10.tocsr() @ AinvB).tocsr()
    Sp = (A11.tocsr() - S).tocsr()
    Sp.sort_indices()
    return Sp


class _SchurOp:
    """S x = A11 x - A10 A00^-1 A01 x (MatMult_SchurComplement)."""

    def __init__(self, A00_ksp, A01, A10, A11):
        self.k, self.A01, self.A10, self.A11 = A00_ksp, A01, A10, A11
        self.shape = A11.shape

    def __matmul__(self, x):
        return self.A11 @ x - self.A10 @ self.k.solve(self.A01 @ x)


class PCFieldSplit:
    type = "fieldsplit"

    def __init__(self, M, is0, is1, db, prefix):
        M = M.tocsr()
        self.is0, self.is1 = np.asarray(is0, dtype=np.int64), np.asarray(is1, dtype=np.int64)
        sub = lambda r, c: M[r][:, c].tocsr()
        self.A00, self.A01 = sub(self.is0, self.is0), sub(self.is0, self.is1)
        self.A10, self.A11 = sub(self.is1, self.is0), sub(self.is1, self.is1)
        self.ftype = opt(db, prefix, "pc_fieldsplit_type", "multiplicative")
        p0, p1 = prefix + "fieldsplit_0_", prefix + "fieldsplit_1_"
        if self.ftype in ("additive", "multiplicative"):
            self.k0 = petsc.ksp_from_options(p0, db, self.A00, self.A00, "preonly", "ilu")
            self.k1 = petsc.ksp_from_options(p1, db, self.A11, self.A11, "preonly", "ilu")
        elif self.ftype == "schur":
            self.fact = opt(db, prefix, "pc_fieldsplit_schur_fact_type", "full")
            pre = opt(db, prefix, "pc_fieldsplit_schur_precondition", "a11")
            self.scale = opt(db, prefix, "pc_fieldsplit_schur_scale", -1.0, float)
            if pre == "selfp":
                self.Sp = selfp(self.A00, self.A01, self.A10, self.A11)
            elif pre == "a11":
                self.Sp = self.A11
            else:
                raise NotImplementedError(f"schur precondition '{pre}' is not restated")
            self.k0 = petsc.ksp_from_options(p0, db, self.A00, self.A00, "preonly", "ilu")
            S = _SchurOp(self.k0, self.A01, self.A10, self.A11)
            self.k1 = petsc.ksp_from_options(p1, db, S, self.Sp, "gmres", "ilu")
        else:
            raise NotImplementedError(f"fieldsplit type '{self.ftype}' is not restated")

    def apply(self, x):
        x = np.asarray(x, dtype=np.float64)
        x0, x1 = x[self.is0], x[self.is1]
        if self.ftype == "additive":
            y0, y1 = self.k0.solve(x0), self.k1.solve(x1)
        elif self.ftype == "multiplicative":
            y0 = self.k0.solve(x0)
            y1 = self.k1.solve(x1 - self.A10 @ y0)
        elif self.fact == "diag":
            y0 = self.k0.solve(x0)
            y1 = self.scale * self.k1.solve(x1)
        elif self.fact == "lower":
            y0 = self.k0.solve(x0)
            y1 = self.k1.solve(x1 - self.A10 @ y0)
        elif self.fact == "upper":
            y1 = self.k1.solve(x1)
            y0 = self.k0.solve(x0 - self.A01 @ y1)
        elif self.fact == "full":
            t = self.k0.solve(x0)
            y1 = self.k1.solve(x1 - self.A10 @ t)
            y0 = self.k0.solve(x0 - self.A01 @ y1)
        else:
            raise NotImplementedError(f"schur fact type '{self.fact}' is not restated")
        y = np.empty_like(x)
        y[self.is0], y[self.is1] = y0, y1
        return y
