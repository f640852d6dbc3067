"""Block preconditioner restatement (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Follows the reference ``lib/Preconditioner.py``:

* sub-blocks of **P** by ``createSubMatrix(isrow, iscol)`` (rows in isrow order,
  columns in iscol order) -- ``allocate_submatrices`` 60-75;
* inner KSPs with prefixes ``s_ f_ p_ diff_ fp_``, ``setType(inner ksp type)``,
  ``pc.setType(inner pc type)`` then ``setFromOptions`` (options win), inner
  tolerances left at PETSc defaults (the stored inner rtol/atol/maxiter are
  never applied: ``__init__`` 22-27 vs ``setup_elliptic_solver`` 94-100);
  ``fp_`` is an elliptic solver when inner pc type is ``lu``, otherwise GMRES +
  fieldsplit (``setUp`` 134-138, ``setup_fieldsplit`` 102-118; oracle/fieldsplit.py);
* ``apply`` 141-250:
  - 2-way: y_s = K_s^-1 x_s ; y_fp = K_fp^-1 (x_fp - P_fp,s y_s)       (221-234)
  - 3-way: FS sweep p -> f -> s and DIFF sweep (pressure-BC rows of x_p zeroed,
    K_p,diff from P_diff), y = w1 y_FS + w2 y_DIFF with w1 = 1, w2 = 0.1
    (150-218; the temporaries are copies: x is never written back);
  - inner Anderson mixing of y when ``inner accel order > 0`` (248-249).
* the factory's pc-type validation and ``flag_3_way`` (263-291).
"""
from __future__ import annotations

import numpy as np

from . import petsc
from .aar import AndersonAcceleration
from .options import get as opt

PC_TYPES = ("undrained", "undrained 3-way", "diagonal", "diagonal 3-way", "diagonal 3-way-II", "lu")


def submatrix(M, isrow, iscol):
    return M[np.asarray(isrow)][:, np.asarray(iscol)].tocsr()


class BlockPC:
    def __init__(self, P, P_diff, index_sets, dims, flag_3_way, db,
                 inner_ksp_type="gmres", inner_pc_type="lu", w1=1.0, w2=0.1,
                 accel_order=0, bcs_sub_pressure=(), dist_size=1, dist_owner=None):
        """dist_size=G: the G-rank preconditioner libpls builds on a synthetic
        field-major system (even slabs per field, oracle/dist.py);
        dist_owner: the rank of every global row of a caller-assembled system
        (pls_create_dist): each block's rows split by owner."""
        self.flag_3_way = flag_3_way
        self.w1, self.w2 = w1, w2
        self.ns, self.nf, self.np = dims
        self.is_s, self.is_f, self.is_p, self.is_fp = [np.asarray(i, dtype=np.int64) for i in index_sets]
        self.bcs = np.asarray(bcs_sub_pressure, dtype=np.int64)
        self.anderson = AndersonAcceleration(accel_order)
        sizes = (self.ns, self.nf, self.np)

        if dist_owner is not None:
            dist_owner = np.asarray(dist_owner)
            dist_size = int(dist_owner.max()) + 1

        def inner(prefix, M, ksp_type, pc_type, fields, rows=None):
            # G ranks: BJACOBI blocks live inside each rank's [field slabs] rows
            # (oracle/dist.py); every other PC type acts on the whole block --
            # libpls gathers it and applies the PC redundantly (PETSc's
            # PCREDUNDANT), so it is the same PC at any G
            pc = None
            if dist_size > 1:
                ptype = opt(db, prefix, "pc_type", pc_type)
                if ptype == "hypre" and str(db.get("pls.hypre", "boomeramg")) == "boomeramg":
                    # BoomerAMG under mpirun -np G: the block's rank partition when every
                    # rank's rows are one contiguous range (single-field slabs, or
                    # caller-assembled ownership) -- libpls runs that np = G hierarchy
                    # with each rank smoothing its own rows (or, pls.hypre_dist 0,
                    # gathered and applied redundantly): the same operator either way
                    sizes_r = None
                    if dist_owner is not None:
                        own = dist_owner[rows]
                        if np.all(np.diff(own) >= 0):
                            sizes_r = np.bincount(own, minlength=dist_size).tolist()
                    elif len(fields) == 1:
                        from .dist import slab
                        sizes_r = [slab(sizes[fields[0]], dist_size, q)[1] for q in range(dist_size)]
                    if sizes_r is not None and "pls.hypre_ranks" not in db:
                        db_r = dict(db, **{"pls.hypre_ranks": ",".join(str(v) for v in sizes_r)})
                        pc = petsc.make_pc_of_type("hypre", M, db_r, prefix)
                if ptype == "bjacobi":
                    from .dist import PCBJacobiIndexed, bjacobi_blocks, bjacobi_blocks_owned
                    nbt = opt(db, prefix, "pc_bjacobi_blocks", dist_size, int)
                    blocks = (bjacobi_blocks_owned(dist_owner[rows], dist_size, nbt) if dist_owner is not None
                              else bjacobi_blocks(sizes, fields, dist_size, nbt))
                    pc = PCBJacobiIndexed(M, blocks, opt(db, prefix + "sub_", "pc_type", "ilu"))
            return petsc.ksp_from_options(prefix, db, M, M, ksp_type, pc_type, pc=pc)

        Ms_s = submatrix(P, self.is_s, self.is_s)
        self.ksp_s = inner("s_", Ms_s, inner_ksp_type, inner_pc_type, (0,), self.is_s)
        if flag_3_way:
            self.Ms_f = submatrix(P, self.is_s, self.is_f)
            self.Ms_p = submatrix(P, self.is_s, self.is_p)
            self.Mf_p = submatrix(P, self.is_f, self.is_p)
            Mf_f = submatrix(P, self.is_f, self.is_f)
            Mp_p = submatrix(P, self.is_p, self.is_p)
            Mp_diff = submatrix(P_diff, self.is_p, self.is_p)
            self.ksp_f = inner("f_", Mf_f, inner_ksp_type, inner_pc_type, (1,), self.is_f)
            self.ksp_p = inner("p_", Mp_p, inner_ksp_type, inner_pc_type, (2,), self.is_p)
            self.ksp_p_diff = inner("diff_", Mp_diff, inner_ksp_type, inner_pc_type, (2,), self.is_p)
        else:
            self.Mfp_s = submatrix(P, self.is_fp, self.is_s)
            Mfp_fp = submatrix(P, self.is_fp, self.is_fp)
            if inner_pc_type == "lu":
                self.ksp_fp = inner("fp_", Mfp_fp, inner_ksp_type, "lu", (1, 2), self.is_fp)
            else:
                # setup_fieldsplit: GMRES + fieldsplit unless the options override the pc type
                ptype = opt(db, "fp_", "pc_type", "fieldsplit")
                if ptype == "fieldsplit":
                    # setFieldSplitIS((None, is_p)) then ((None, is_f)): split 0 = pressure
                    from .fieldsplit import PCFieldSplit
                    # G ranks: the gathered fp block, redundantly (same PC at any G)
                    fs = PCFieldSplit(Mfp_fp, self.is_p, self.is_f, db, "fp_")
                    self.ksp_fp = petsc.ksp_from_options("fp_", db, Mfp_fp, Mfp_fp, "gmres", "fieldsplit", pc=fs)
                else:
                    self.ksp_fp = inner("fp_", Mfp_fp, "gmres", ptype, (1, 2), self.is_fp)

    def apply(self, x):
        x = np.asarray(x, dtype=np.float64)
        y = np.zeros_like(x)
        x_s = x[self.is_s]
        if self.flag_3_way:
            x_f = x[self.is_f]
            x_p = x[self.is_p]
            y_p = self.ksp_p.solve(x_p)
            x_pd = x_p.copy()
            x_pd[self.bcs] = 0.0
            y_pd = self.ksp_p_diff.solve(x_pd)
            t_f = x_f - self.Mf_p @ y_p
            y_f = self.ksp_f.solve(t_f)
            t_f = x_f - self.Mf_p @ y_pd
            y_fd = self.ksp_f.solve(t_f)
            t_s = x_s - (self.Ms_f @ y_f + self.Ms_p @ y_p)
            y_s = self.ksp_s.solve(t_s)
            t_s = x_s - (self.Ms_f @ y_fd + self.Ms_p @ y_pd)
            y_sd = self.ksp_s.solve(t_s)
            y[self.is_p] = self.w1 * y_p + self.w2 * y_pd
            y[self.is_f] = self.w1 * y_f + self.w2 * y_fd
            y[self.is_s] = self.w1 * y_s + self.w2 * y_sd
        else:
            y_s = self.ksp_s.solve(x_s)
            t = x[self.is_fp] - self.Mfp_s @ y_s
            y_fp = self.ksp_fp.solve(t)
            y[self.is_s] = y_s
            y[self.is_fp] = y_fp
        if self.anderson.order > 0:
            y = self.anderson.get_next_vector(y)
        return y


def make_block_pc(P, P_diff, index_sets, dims, parameters, db, bcs_sub_pressure, dist_size=1, dist_owner=None):
    """Preconditioner(...).get_pc() restated (lib/Preconditioner.py:263-291)."""
    pc_type = parameters["pc type"]
    if pc_type not in PC_TYPES:
        raise SystemExit("pc type must be one of lu, undrained, diagonal, diagonal 3-way, diagonal 3-way-II.")
    flag_3_way = pc_type in ("diagonal 3-way", "undrained 3-way")
    return BlockPC(P, P_diff, index_sets, dims, flag_3_way, db,
                   parameters["inner ksp type"], parameters["inner pc type"], 1.0, 0.1,
                   parameters["inner accel order"], bcs_sub_pressure, dist_size, dist_owner)
