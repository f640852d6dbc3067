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
* static pivoting (opt-in since round 6, MUMPS's CNTL(4) default): a block
  with an exactly singular pivot (a zeroed row and column) factors with the
  pivot replaced by tau when pls.lu_static_pivot is set (the apply is
  finite), and is PETSc's MAT_FACTOR_NUMERIC_ZEROPIVOT error by default;
* threshold partial pivoting over each front's fully-summed rows (MUMPS
  CNTL(1) = 0.01): a block whose leading tile is exactly zero.
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
    h = _handle(s, {"pls.lu_static_pivot": str(64 * 2.220446049250313e-16)}, P=P)  # opt-in (MUMPS CNTL(4) > 0)
    y = h.pc_apply(x)
    h.destroy()
    assert np.all(np.isfinite(y))
    with pytest.raises(RuntimeError, match="zero pivot"):
        h = _handle(s, {}, P=P)  # default: off, an exactly singular block is an error (MUMPS: INFO(1) = -10)
        try:
            h.pc_apply(x)
        finally:
            h.destroy()


def _swap_system(n2=64, eps=0.05):
    """A 3-field system whose solid block K = [[0, B], [B^T, 0]] (B = I + eps
    tridiag, 2 n2 rows) has an exactly zero leading 64 x 64 tile: LU without
    pivoting fails at its first pivot, LU with row exchanges does not (K is
    nonsingular, det = det(B)^2 up to sign).  Fluid and pressure blocks:
    identity, no coupling -- the 2-way PC's y is [K^-1 x_s, x_fp]."""
    import types
    B = sp.eye(n2) + eps * sp.diags([np.ones(n2 - 1), np.ones(n2 - 1)], [-1, 1])
    K = sp.bmat([[None, B], [B.T, None]]).tocsr()
    ns, nf, npr = 2 * n2, 32, 32
    P = sp.block_diag([K, sp.eye(nf), sp.eye(npr)]).tocsr()
    P.sort_indices()
    n = P.shape[0]
    s = types.SimpleNamespace(A=P, P=P, P_diff=None, is_s=np.arange(ns, dtype=np.int32),
                              is_f=np.arange(ns, ns + nf, dtype=np.int32),
                              is_p=np.arange(ns + nf, n, dtype=np.int32), bcs_sub_pressure=[])
    return s, K


def _swap_apply(s, extra):
    from lib.handle import Handle, params_to_options
    opts = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "s_ksp_type": "preonly", "s_pc_type": "lu",
            "fp_ksp_type": "preonly", "fp_pc_type": "lu", "pls.lu_view": "1"}
    opts.update(extra)
    opts.update(params_to_options(BASE))
    h = Handle.from_csr(s.A, s.P, None, s.is_s, s.is_f, s.is_p, s.bcs_sub_pressure, opts)
    try:
        x = np.random.default_rng(8).standard_normal(s.A.shape[0])
        return x, h.pc_apply(x)
    finally:
        h.destroy()


@pytest.mark.parametrize("path", ["dense", "sparse"])
def test_lu_threshold_pivoting_zero_leading_tile(gpu, capfd, path):
    """MUMPS's threshold partial pivoting (CNTL(1) = u = 0.01, pls.lu_pivot_threshold):
    each 64 x 64 tile's pivots are chosen over all the front's remaining
    fully-summed rows (the dense path: all remaining rows), so the zero leading
    tile takes its pivots from the other half; the exact solve against numpy.
    Without it (u = 0) the same block is a zero pivot -- static pivoting is off
    by default as in MUMPS (CNTL(4) <= 0)."""
    import scipy.sparse.linalg as spla
    s, K = _swap_system()
    extra = {"pls.lu_path": path, "pls.lu_nd_leaf": "256", "pls.lu_nd_compress": "0"}
    capfd.readouterr()
    x, y = _swap_apply(s, extra)
    err = capfd.readouterr().err
    ns = K.shape[0]
    ys = spla.spsolve(K.tocsc(), x[:ns])
    assert np.max(np.abs(y[:ns] - ys)) <= 1e-12 * np.max(np.abs(ys))
    assert np.array_equal(y[ns:], x[ns:])
    line = [l for l in err.splitlines() if ("[sparse lu] n %d" % ns if path == "sparse" else "[dense lu] n %d" % ns) in l]
    assert line and " 0 rows exchanged" not in line[0], err
    with pytest.raises(RuntimeError, match="zero pivot"):
        _swap_apply(s, dict(extra, **{"pls.lu_pivot_threshold": "0"}))


def test_lu_delayed_pivot(gpu, capfd):
    """A pivot MUMPS must delay (petsc-options-exact:11-35's LU): 4 disjoint
    stars, center s (diagonal 4) coupled by 1 to leaves a1 (diagonal 1e-14)
    and a2, a3, a4 (diagonal 2) -- nonsingular.  The dissection (leaves of one
    vertex, ``sparse_lu_analyze``) puts {a1, a3} in one leaf front and s in its
    parent: a1's column has the fully-summed entry 1e-14 against the update
    row's 1, below u = 0.01 of the column, so it is delayed to the parent
    front, where rows s and a1 are both fully summed and the exchange picks s.
    Solved to rounding against numpy; with the delays off
    (pls.lu_delay_rounds 0) the 1e-14 pivot is used and the solve loses
    ~1e14 x 1e-16 of its accuracy."""
    import types

    import scipy.sparse.linalg as spla
    from lib.handle import sparse_lu_analyze
    star = np.array([[4, 1, 1, 1, 1], [1, 1e-14, 0, 0, 0], [1, 0, 2, 0, 0], [1, 0, 0, 2, 0], [1, 0, 0, 0, 2]], float)
    K = sp.block_diag([sp.csr_matrix(star)] * 4).tocsr()
    nd = {"pls.lu_nd_leaf": "1", "pls.lu_nd_compress": "0"}
    _, perm, front_of, parent = sparse_lu_analyze(K, nd, tree=True)
    pos = {int(v): k for k, v in enumerate(perm)}
    assert front_of[pos[1]] != front_of[pos[0]] and parent[front_of[pos[1]]] == front_of[pos[0]]  # a1 below s
    ns, nf, npr = K.shape[0], 8, 8
    P = sp.block_diag([K, sp.eye(nf), sp.eye(npr)]).tocsr()
    P.sort_indices()
    s = types.SimpleNamespace(A=P, P=P, P_diff=None, is_s=np.arange(ns, dtype=np.int32),
                              is_f=np.arange(ns, ns + nf, dtype=np.int32),
                              is_p=np.arange(ns + nf, P.shape[0], dtype=np.int32), bcs_sub_pressure=[])
    extra = dict(nd, **{"pls.lu_path": "sparse"})
    capfd.readouterr()
    x, y = _swap_apply(s, extra)
    err = capfd.readouterr().err
    ys = spla.spsolve(K.tocsc(), x[:ns])
    assert np.max(np.abs(y[:ns] - ys)) <= 1e-12 * np.max(np.abs(ys)), np.max(np.abs(y[:ns] - ys))
    line = [l for l in err.splitlines() if "[sparse lu] n %d" % ns in l]
    assert line and " 4 delayed pivots" in line[0], err
    x2, y2 = _swap_apply(s, dict(extra, **{"pls.lu_delay_rounds": "0"}))
    assert np.max(np.abs(y2[:ns] - ys)) > 1e-8 * np.max(np.abs(ys))  # the 1e-14 pivot, undelayed
