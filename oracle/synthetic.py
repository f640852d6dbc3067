"""Seeded synthetic 3-field block system; TEST INFRASTRUCTURE ONLY.

The reference assembles A, P, P_diff with dolfin (reference
``lib/Assembler.py:66-221``) -- not available here.  The synthetic stand-in keeps
the structure the solver path sees:

* fields s (solid displacement), f (fluid velocity), p (pressure) with the
  P2^d x P2^d x P1 sizes of the reference meshes (``lib/Poromechanics.py:14-18``):
  3-D ns = nf = 3(2N+1)^3, np = (N+1)^3; 2-D ns = nf = 2(2N+1)^2, np = (N+1)^2;
* a symmetric banded pattern per field block (offset stencils drawn once per
  block inside a band W that mimics a bandwidth-reduced FE ordering) with about
  the per-row counts of the dolfin mixed-space sparsity (~182 nnz/row in 3-D);
* symmetric values, off-diagonals U(-1,0) (x0.1 across fields, B_fs = B_sf^T),
  diagonal = sum |off-diag| + delta (1 + U(0,1)): SPD, strictly diagonally
  dominant, an M-matrix (ILU(0) exists);
* P = A except its diagonal draw; P_diff = P with the pressure Dirichlet rows
  (``bcs_sub_pressure``, ``lib/Poromechanics.py:48-55``) replaced by identity rows.

The C kernel (oracle/csrc/oracle.c) is the definition; the HIP generator of
the product must reproduce it bit for bit.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp

from . import native

VARIANT_A, VARIANT_P, VARIANT_PDIFF = 0, 1, 2
DEFAULT_SEED = 20261015
DEFAULT_DELTA = 0.05

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    z = (z + np.uint64(0x9E3779B97F4A7C15)) & _M
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M
    return z ^ (z >> np.uint64(31))


def _hash3(s, a, b):
    with np.errstate(over="ignore"):
        return _mix64(_mix64(_mix64(np.uint64(s)) ^ np.asarray(a, dtype=np.uint64))
                      ^ np.asarray(b, dtype=np.uint64))


@dataclass(frozen=True)
class SynthSpec:
    dim: int = 3
    N: int = 4
    seed: int = DEFAULT_SEED
    delta: float = DEFAULT_DELTA

    def sizes(self):
        out = np.zeros(9, dtype=np.int64)
        rc = native.lib().oracle_synth_sizes(self.dim, self.N, self.seed, out)
        if rc:
            raise ValueError(f"bad synthetic spec {self} (rc={rc})")
        return int(out[0]), int(out[1]), int(out[2])

    @property
    def n(self):
        return sum(self.sizes())

    def offsets(self, block: int):
        out = np.zeros(128, dtype=np.int32)
        m = native.lib().oracle_synth_offsets(self.dim, self.N, self.seed, block, out)
        return out[:m].copy()


def matrix(spec: SynthSpec, variant: int = VARIANT_A) -> sp.csr_matrix:
    """Full n x n CSR in field-major order [s | f | p]."""
    L = native.lib()
    n = spec.n
    rp = np.zeros(n + 1, dtype=np.int64)
    if L.oracle_synth_rowptr(spec.dim, spec.N, spec.seed, rp):
        raise ValueError("synth rowptr failed")
    nnz = int(rp[-1])
    ci = np.zeros(nnz, dtype=np.int32)
    v = np.zeros(nnz, dtype=np.float64)
    if L.oracle_synth_fill(spec.dim, spec.N, spec.seed, spec.delta, variant, rp, ci, v):
        raise ValueError("synth fill failed")
    M = sp.csr_matrix((v, ci, rp), shape=(n, n))
    M.has_sorted_indices = True
    return M


def rhs(spec: SynthSpec) -> np.ndarray:
    b = np.zeros(spec.n, dtype=np.float64)
    native.lib().oracle_synth_rhs(spec.seed, spec.n, b)
    return b


def bcs_sub_pressure(spec: SynthSpec) -> np.ndarray:
    """Positions inside the p sub-vector that carry a pressure Dirichlet BC."""
    np_ = spec.sizes()[2]
    i = np.arange(np_, dtype=np.uint64)
    h = _hash3(np.uint64(spec.seed) ^ np.uint64(0x00BC00), i, np.uint64(7))
    return np.nonzero((h & np.uint64(15)) == 0)[0].astype(np.int32)


def field_major_index_sets(spec: SynthSpec):
    ns, nf, np_ = spec.sizes()
    is_s = np.arange(0, ns, dtype=np.int32)
    is_f = np.arange(ns, ns + nf, dtype=np.int32)
    is_p = np.arange(ns + nf, ns + nf + np_, dtype=np.int32)
    return is_s, is_f, is_p


def interleaving(spec: SynthSpec):
    """A dolfin-like interleaved dof order.

    Returns ``perm`` with ``perm[new] = old`` (old = field-major index): dofs of
    the three fields are merged by their normalised position i / n_field, so
    each field keeps its internal order and the index sets are non-contiguous,
    as dolfin's mixed-space dofmaps are (reference ``lib/IndexSet.py:38-41``).
    """
    ns, nf, np_ = spec.sizes()
    keys = np.concatenate([(np.arange(ns) + 0.25) / ns,
                           (np.arange(nf) + 0.50) / nf,
                           (np.arange(np_) + 0.75) / np_])
    return np.argsort(keys, kind="stable").astype(np.int64)


def permute(M: sp.csr_matrix, perm: np.ndarray) -> sp.csr_matrix:
    """Symmetric permutation: B[new_i, new_j] = M[perm[new_i], perm[new_j]]."""
    B = M[perm][:, perm].tocsr()
    B.sort_indices()
    return B


def index_sets_for(perm: np.ndarray, spec: SynthSpec):
    """Global (sorted) index sets of each field in the permuted ordering."""
    ns, nf, np_ = spec.sizes()
    inv = np.empty_like(perm)
    inv[perm] = np.arange(perm.size)
    is_s = np.sort(inv[:ns]).astype(np.int32)
    is_f = np.sort(inv[ns:ns + nf]).astype(np.int32)
    is_p = np.sort(inv[ns + nf:]).astype(np.int32)
    return is_s, is_f, is_p
