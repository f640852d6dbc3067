"""Distributed-solve restatement (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

The reference runs with MPI data parallelism (``mpirun -np 8``,
paper-scripts/robustness_2d.sh:29): PETSc MPIAIJ row ownership, halo
VecScatters in MatMult, MPI_Allreduce in dots/norms, and BJACOBI inner blocks
that live inside one rank's diagonal block.  libpls.so shards the same way
(DESIGN.md §6): rank r owns a PETSc-split slab of every field, its local
vectors are [s_r | f_r | p_r], and a field block's inner BJACOBI splits the
*rank-local* rows into B / G (+1 for the first B % G ranks) blocks.

This module gives
* the partition (``slab``, ``local_rows``) -- same split as the library;
* ``PCBJacobiIndexed``: block Jacobi over explicit index blocks, so the
  single-process oracle can run exactly the G-rank preconditioner;
* ``bjacobi_blocks(sizes, fields, G, B)``: the per-rank blocks of a field
  block (fp: each rank's [f_r | p_r] rows, in that order).
"""
from __future__ import annotations

import numpy as np

from . import petsc


def slab(n: int, size: int, r: int):
    q, rem = divmod(n, size)
    lo = r * q + min(r, rem)
    return lo, q + (1 if r < rem else 0)


def local_rows(sizes, size, r):
    """Global field-major rows owned by rank r, in local order [s_r | f_r | p_r]."""
    off = np.concatenate([[0], np.cumsum(sizes)])
    parts = []
    for f in range(3):
        lo, ln = slab(sizes[f], size, r)
        parts.append(off[f] + lo + np.arange(ln))
    return np.concatenate(parts).astype(np.int64)


def bjacobi_blocks(sizes, fields, size, total_blocks):
    """Index blocks (into the field-block matrix) of BJACOBI over G ranks."""
    off = np.concatenate([[0], np.cumsum([sizes[f] for f in fields])])
    blocks = []
    for r in range(size):
        loc = np.concatenate([off[i] + slab(sizes[f], size, r)[0] + np.arange(slab(sizes[f], size, r)[1])
                              for i, f in enumerate(fields)]).astype(np.int64)
        nb = max(1, total_blocks // size + (1 if r < total_blocks % size else 0))
        lens = petsc.bjacobi_block_sizes(len(loc), nb)
        b0 = 0
        for ln in lens:
            blocks.append(loc[b0:b0 + ln])
            b0 += ln
    return blocks


def bjacobi_blocks_owned(owner, size, total_blocks):
    """BJACOBI blocks of a field block whose row i lives on rank owner[i] (a
    caller-assembled system: PETSc's createSubMatrix keeps each rank's own IS
    entries, so rank r's rows are the block rows it owns, in block order)."""
    owner = np.asarray(owner)
    blocks = []
    for r in range(size):
        loc = np.nonzero(owner == r)[0].astype(np.int64)
        nb = max(1, total_blocks // size + (1 if r < total_blocks % size else 0))
        lens = petsc.bjacobi_block_sizes(len(loc), nb) if len(loc) else []
        b0 = 0
        for ln in lens:
            blocks.append(loc[b0:b0 + ln])
            b0 += ln
    return blocks


def row_owner(n, size):
    """Rank of each global row under PETSc's default MPIAIJ split of n rows."""
    own = np.empty(n, dtype=np.int64)
    for r in range(size):
        lo, ln = slab(n, size, r)
        own[lo:lo + ln] = r
    return own


class PCBJacobiIndexed:
    type = "bjacobi"

    def __init__(self, M, blocks, sub_pc_type="ilu"):
        M = M.tocsr()
        self.blocks = blocks
        self.subs = [petsc.make_pc_of_type(sub_pc_type, M[idx][:, idx].tocsr()) for idx in blocks]

    def apply(self, x):
        y = np.empty_like(x)
        for idx, s in zip(self.blocks, self.subs):
            y[idx] = s.apply(x[idx])
        return y


FIELDS_OF_PREFIX_2WAY = {"s_": (0,), "fp_": (1, 2)}
FIELDS_OF_PREFIX_3WAY = {"s_": (0,), "f_": (1,), "p_": (2,), "diff_": (2,)}


# ------------------------------------------------ G-rank emulation (gloo) --
# One process per rank, each holding only its rows, exactly as libpls shards
# the solve: SpMV over a gathered input vector (the library exchanges only the
# halo entries it needs -- same products), inner products as the rank-ordered
# sum of per-rank partials (Comm::global_sum_dev), block Jacobi inside the
# rank's rows.  tests/test_dist_cpu.py checks it against the single-process
# ``OracleSolver(dist_size=G)`` -- the decomposition argument behind comparing
# G GPU ranks with that oracle.

class GlooComm:
    """allgather over torch.distributed (any backend with CPU tensors, e.g. gloo)."""

    def __init__(self):
        import torch.distributed as td
        self.td = td
        self.rank, self.size = td.get_rank(), td.get_world_size()

    def allgather(self, a):
        import torch
        a = np.ascontiguousarray(a, dtype=np.float64).ravel()
        n = torch.tensor([a.size], dtype=torch.int64)
        ns = [torch.zeros(1, dtype=torch.int64) for _ in range(self.size)]
        self.td.all_gather(ns, n)
        mx = max(int(t) for t in ns)
        buf = torch.zeros(mx, dtype=torch.float64)
        buf[:a.size] = torch.from_numpy(a)
        out = [torch.zeros(mx, dtype=torch.float64) for _ in range(self.size)]
        self.td.all_gather(out, buf)
        return [o.numpy()[:int(k)].copy() for o, k in zip(out, ns)]

    def global_sum(self, vals):
        s = np.zeros(np.asarray(vals).size)
        for part in self.allgather(vals):
            s = s + part
        return s


class DistKSP(petsc.KSP):
    comm = None

    def dot(self, a, b):
        return float(self.comm.global_sum([np.dot(a, b)])[0])

    def norm(self, a):
        return float(np.sqrt(self.comm.global_sum([np.dot(a, a)])[0]))


def _distribute(ksp, comm):
    ksp.__class__ = DistKSP
    ksp.comm = comm
    return ksp


class RankSolver2Way:
    """Rank r's share of Solver(gmres / 2-way block PC) on the field-major system."""

    def __init__(self, A, P, sizes, parameters, db, comm):
        from .options import get as opt
        self.comm = comm
        G, r = comm.size, comm.rank
        self.sizes = sizes
        off = np.concatenate([[0], np.cumsum(sizes)])
        self.rows = [local_rows(sizes, G, q) for q in range(G)]
        L = self.rows[r]
        ls = slab(sizes[0], G, r)[1]
        self.ls = ls
        s_rows, fp_rows = L[:ls], L[ls:]
        s_all = np.arange(off[0], off[1])
        A, P = A.tocsr(), P.tocsr()
        self.A_loc = A[L]                      # local rows, global columns
        self.Mfp_s = P[fp_rows][:, s_all]      # global s columns
        self.s_parts = [self.rows[q][:slab(sizes[0], G, q)[1]] for q in range(G)]

        def inner(prefix, M, pc_type):
            ptype = opt(db, prefix, "pc_type", pc_type)
            pc = None
            if ptype == "bjacobi":
                nbt = opt(db, prefix, "pc_bjacobi_blocks", G, int)
                nb = max(1, nbt // G + (1 if r < nbt % G else 0))
                pc = petsc.PCBJacobi(M, nb, opt(db, prefix + "sub_", "pc_type", "ilu"))
            return _distribute(petsc.ksp_from_options(prefix, db, M, M, parameters["inner ksp type"],
                                                      pc_type, pc=pc), comm)

        ipt = parameters["inner pc type"]
        self.ksp_s = inner("s_", P[s_rows][:, s_rows], ipt)
        self.ksp_fp = inner("fp_", P[fp_rows][:, fp_rows], "lu" if ipt == "lu" else opt(db, "fp_", "pc_type", "fieldsplit"))
        self.n_glob = int(off[-1])
        outer_pc = petsc.PCShell(self.pc_apply)
        stype = parameters["solver type"]
        maxiter = parameters["solver maxiter"]
        self.ksp = _distribute(petsc.ksp_from_options(
            "global_", db, None, None, stype, "python", rtol=parameters["solver rtol"],
            atol=parameters["solver atol"], dtol=1e20, maxit=maxiter,
            restart=maxiter if stype == "gmres" else petsc.GMRES_DEFAULT_RESTART, pc=outer_pc), comm)
        self.ksp.matvec = self.matvec

    def _gather_global(self, x_loc, parts_rows, n):
        out = np.zeros(n)
        for rows, piece in zip(parts_rows, self.comm.allgather(x_loc)):
            out[rows] = piece
        return out

    def matvec(self, x_loc):
        return self.A_loc @ self._gather_global(x_loc, self.rows, self.n_glob)

    def pc_apply(self, x_loc):
        ls = self.ls
        y_s = self.ksp_s.solve(x_loc[:ls])
        y_s_glob = self._gather_global(y_s, self.s_parts, self.sizes[0])
        y_fp = self.ksp_fp.solve(x_loc[ls:] - self.Mfp_s @ y_s_glob)
        return np.concatenate([y_s, y_fp])

    def solve(self, b_loc):
        return self.ksp.solve(b_loc)
