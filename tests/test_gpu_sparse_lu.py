"""The sparse LU (the MUMPS stand-in, csrc/sparse_lu.cpp; petsc-options-exact:
11-35, petsc-options-inexact:105-106) forced onto small assembled blocks.

* the 2-way "diagonal" block PC with PREONLY + LU on K_s and on the
  saddle-point fp block (zero pressure diagonals) through the
  sparse path with ND leaves of 8 and 64 rows: ||K y - x|| / ||x|| against the
  blocks exported from the handle, unrefined (pls.lu_refine 0) and refined.
  The bound for the ill-conditioned undrained solid block is LAPACK's own
  level: dense partial-pivoting LU (scipy lu_factor + lu_solve) leaves
  4.1e-11 (N=8) .. 4.7e-11 (N=16) on it, so unrefined <= 1e-9, refined
  <= 2e-10; the fp block is well conditioned: <= 1e-12 either way;
* static pivoting: a block with an exactly singular pivot (a zeroed row and
  column) factors with the pivot replaced by tau (the apply is finite), and
  pls.lu_static_pivot 0 restores PETSc's MAT_FACTOR_NUMERIC_ZEROPIVOT error.
"""
import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu

BASE = {"solver type": "gmres", "solver atol": 1e-10, "solver rtol": 1e-8, "solver maxiter": 50,
        "pc type": "diagonal", "inner ksp type": "preonly", "inner pc type": "lu", "inner accel order": 0,
        "AAR order": 10, "AAR p": 5, "AAR omega": 1, "AAR beta": 1}


def _handle(s, extra, P=None):
    from lib.handle import Handle, params_to_options
    db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "s_ksp_type": "preonly", "s_pc_type": "lu",
          "fp_ksp_type": "preonly", "fp_pc_type": "lu", "pls.lu_path": "sparse"}
    db.update(extra)
    opts = dict(db)
    opts.update(params_to_options(BASE))
    return Handle.from_csr(s.A, s.P if P is None else P, None, s.is_s, s.is_f, s.is_p, [], opts)


def _block_residuals(s, y, x, P=None):
    """||(M y - x)_s|| / ||x_s||, same for fp; M = P with its s-rows / fp-columns block dropped."""
    P = (s.P if P is None else P).tocoo()
    n = P.shape[0]
    ins = np.zeros(n, bool)
    ins[s.is_s] = True
    keep = ~(ins[P.row] & ~ins[P.col])
    M = sp.csr_matrix((P.data[keep], (P.row[keep], P.col[keep])), shape=P.shape)
    r = M @ y - x
    fp = np.concatenate([s.is_f, s.is_p])
    return (np.linalg.norm(r[s.is_s]) / np.linalg.norm(x[s.is_s]),
            np.linalg.norm(r[fp]) / np.linalg.norm(x[fp]))


@pytest.mark.parametrize("leaf", ["8", "64"])
@pytest.mark.parametrize("system", ["footing8", "swelling2d8"])
def test_sparse_lu_on_fe_blocks(gpu, system, leaf):
    if system == "footing8":
        from lib.fe_footing import assemble_footing
        s = assemble_footing(8, "undrained")
    else:
        from lib.fe_swelling import assemble_swelling
        s = assemble_swelling(2, 8, "diagonal")
    x = np.random.default_rng(5).standard_normal(s.A.shape[0])
    for refine, bound_s in (("0", 1e-9), ("1", 2e-10)):
        h = _handle(s, {"pls.lu_nd_leaf": leaf, "pls.lu_refine": refine})
        y = h.pc_apply(x)
        h.destroy()
        rs, rfp = _block_residuals(s, y, x)
        assert rs <= bound_s, (system, leaf, refine, rs)
        assert rfp <= 1e-12, (system, leaf, refine, rfp)


def test_sparse_lu_static_pivot(gpu):
    from lib.fe_swelling import assemble_swelling
    s = assemble_swelling(2, 8, "diagonal")
    P = s.P.tocsr().copy()
    P.sort_indices()
    z = int(s.is_s[len(s.is_s) // 2])
    rows = np.repeat(np.arange(P.shape[0]), np.diff(P.indptr))
    P.data[(rows == z) | (P.indices == z)] = 0.0  # row and column z zero, structure (and its diagonal) kept
    x = np.random.default_rng(6).standard_normal(s.A.shape[0])
    h = _handle(s, {}, P=P)
    y = h.pc_apply(x)
    h.destroy()
    assert np.all(np.isfinite(y))
    with pytest.raises(RuntimeError, match="zero pivot"):
        h = _handle(s, {"pls.lu_static_pivot": "0"}, P=P)
        try:
            h.pc_apply(x)
        finally:
            h.destroy()
