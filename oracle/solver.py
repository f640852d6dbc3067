"""Outer solver flow restated (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Follows the reference:
* ``lib/IndexSet.py:10-26,46-54``: in 2-way mode is_f / is_p are re-indexed to
  their positions inside the sorted fp set;
* ``lib/Solver.py:64-103``: KSP with prefix ``global_``, ``setType(solver
  type)``, ``setTolerances(rtol, atol, 1e20, maxiter)``, GMRES restart = maxiter,
  then ``setFromOptions``; or ``AAR(order, p, omega, beta, A, pc, atol, rtol,
  maxiter)`` when solver type is ``aar``;
* ``lib/Poromechanics.py:58-68,88-89``: the PC is built first, then the solver,
  then ``solve(b, x)`` from a zero guess.
"""
from __future__ import annotations

import numpy as np

from . import petsc
from .aar import AAR
from .blockpc import make_block_pc


def local_fp_dofs(dofs_fp_global, dofmap_f, dofmap_p):
    """get_local_fp_dofs (IndexSet.py:10-26): positions of f / p dofs in fp."""
    fset, pset = set(int(d) for d in dofmap_f), set(int(d) for d in dofmap_p)
    dofs_f, dofs_p = [], []
    for i, dof in enumerate(dofs_fp_global):
        if int(dof) in fset:
            dofs_f.append(i)
        elif int(dof) in pset:
            dofs_p.append(i)
    return np.asarray(dofs_f, dtype=np.int32), np.asarray(dofs_p, dtype=np.int32)


def index_sets(is_s, is_f, is_p, two_way):
    """IndexSet.__init__ (IndexSet.py:30-61) on plain integer arrays."""
    is_fp = np.asarray(sorted(list(map(int, is_f)) + list(map(int, is_p))), dtype=np.int32)
    if two_way:
        is_f, is_p = local_fp_dofs(is_fp, is_f, is_p)
    return (np.asarray(is_s, dtype=np.int32), np.asarray(is_f, dtype=np.int32),
            np.asarray(is_p, dtype=np.int32), is_fp)


class OracleSolver:
    def __init__(self, A, P, P_diff, is_s, is_f, is_p, parameters, db, bcs_sub_pressure=(), dist_size=1,
                 dist_owner=None):
        """dist_size=G: the preconditioner libpls builds on G ranks (oracle/dist.py);
        dist_owner: rank of every global row (caller-assembled systems, pls_create_dist)."""
        pc_type = parameters["pc type"]
        two_way = "3-way" not in pc_type
        sets = index_sets(is_s, is_f, is_p, two_way)
        dims = (len(is_s), len(is_f), len(is_p))
        self.block_pc = make_block_pc(P, P_diff, sets, dims, parameters, db, bcs_sub_pressure, dist_size, dist_owner)
        self.pc = petsc.PCShell(self.block_pc.apply)
        stype = parameters["solver type"]
        atol = parameters["solver atol"]
        rtol = parameters["solver rtol"]
        maxiter = parameters["solver maxiter"]
        self.kind = stype
        if stype == "aar":
            self.solver = AAR(parameters["AAR order"], parameters["AAR p"], parameters["AAR omega"],
                              parameters["AAR beta"], A, self.pc, atol=atol, rtol=rtol, maxiter=maxiter)
        else:
            restart = maxiter if stype == "gmres" else petsc.GMRES_DEFAULT_RESTART
            self.solver = petsc.ksp_from_options("global_", db, A, A, stype, "python", rtol=rtol,
                                                 atol=atol, dtol=1e20, maxit=maxiter,
                                                 restart=restart, pc=self.pc)

    def solve(self, b):
        return self.solver.solve(b)

    @property
    def its(self):
        return self.solver.it if self.kind == "aar" else self.solver.its

    @property
    def history(self):
        return self.solver.history

    @property
    def reason(self):
        """KSP reason; for AAR the stop test that ended the loop (AAR.py:73):
        CONVERGED_ATOL (3), CONVERGED_RTOL (2) or DIVERGED_ITS (-3)."""
        if self.kind != "aar":
            return self.solver.reason
        s = self.solver
        h = s.history
        if h[-1] <= s.atol:
            return 3
        if h[-1] / h[0] <= s.rtol:
            return 2
        return -3
