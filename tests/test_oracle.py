"""Known-answer tests that pin the CPU oracle (no GPU).

The reference holds no tests, fixtures or golden vectors and PETSc is not in
this image, so each restated algorithm is pinned against an
independent implementation or a closed-form answer:
  * MatMult            vs scipy ``A @ x``
  * ILU(0)             vs a dense textbook IKJ restatement; = exact LU when no
                       fill is dropped (tridiagonal); hand-computed 3x3
  * MatSolve           vs dense triangular solves of the ILU factors
  * GMRES              residual estimates vs dense least-squares residuals over
                       an explicitly built Krylov basis (left, right, restart);
                       final estimate vs true residual; hand 2x2 case
  * CG                 vs a textbook CG transcription, iteration by iteration
  * KSPConvergedDefault / bjacobi block sizes / options-file parsing / fp index
                       re-mapping: closed-form cases
  * block PC           2-way exact inner == block-lower solve; 3-way FS sweep
                       == block-upper solve, DIFF sweep with BC rows zeroed
  * AAR / Anderson     order 0 == Richardson; an Anderson step's alpha ==
                       lstsq; warm-up pairing quirk traced explicitly
  * synthetic system   symmetric, SPD, diagonally dominant, sizes/nnz per
                       SURVEY.md 8(a), C generator == an independent numpy
                       enumeration of the same spec
"""
import numpy as np
import pytest
import scipy.linalg as sla
import scipy.sparse as sp

from oracle import aar as AA
from oracle import blockpc as BP
from oracle import native, options, petsc
from oracle import synthetic as S
from oracle.solver import OracleSolver, local_fp_dofs


def rand_spd(n, density=0.2, seed=0, shift=0.5):
    rng = np.random.default_rng(seed)
    M = sp.random(n, n, density=density, random_state=rng, format="csr")
    M = -(abs(M) + abs(M).T)
    d = np.asarray(abs(M).sum(axis=1)).ravel() + shift
    M = (M + sp.diags(d)).tocsr()
    M.sort_indices()
    return M


# ------------------------------------------------------------ MatMult / ILU --
def test_spmv_matches_scipy():
    M = rand_spd(300, seed=1)
    x = np.random.default_rng(2).standard_normal(300)
    assert np.allclose(native.spmv(M, x), M @ x, rtol=1e-14, atol=1e-14)


def dense_ilu0(A):
    """Textbook IKJ ILU(0) on a dense array restricted to the pattern of A."""
    A = A.copy()
    n = A.shape[0]
    pat = A != 0
    for i in range(1, n):
        for k in range(i):
            if pat[i, k] and A[i, k] != 0:
                A[i, k] = A[i, k] / A[k, k]
                for j in range(k + 1, n):
                    if pat[i, j] and pat[k, j]:
                        A[i, j] -= A[i, k] * A[k, j]
    return A


def test_ilu0_matches_dense_restatement():
    M = rand_spd(60, density=0.15, seed=3)
    f = native.ILU0(M)
    LU = sp.csr_matrix((f.lu, f.ci, f.rp), shape=M.shape).toarray()
    D = dense_ilu0(M.toarray())
    assert np.allclose(LU[M.toarray() != 0], D[M.toarray() != 0], rtol=1e-13, atol=1e-14)
    assert np.allclose(1.0 / f.dinv, np.diag(D), rtol=1e-14)


def test_ilu0_hand_3x3():
    A = np.array([[4.0, -1.0, 0.0], [-1.0, 4.0, -1.0], [0.0, -1.0, 4.0]])
    f = native.ILU0(sp.csr_matrix(A))
    # exact LU of a tridiagonal matrix: l21 = -1/4, u22 = 15/4, l32 = -4/15, u33 = 56/15
    LU = sp.csr_matrix((f.lu, f.ci, f.rp), shape=(3, 3)).toarray()
    assert np.isclose(LU[1, 0], -0.25) and np.isclose(LU[1, 1], 3.75)
    assert np.isclose(LU[2, 1], -4.0 / 15.0) and np.isclose(LU[2, 2], 56.0 / 15.0)
    b = np.array([1.0, 2.0, 3.0])
    assert np.allclose(f.solve(b), np.linalg.solve(A, b), rtol=1e-14)


def test_ilu0_solve_matches_dense_triangular():
    M = rand_spd(80, density=0.1, seed=4)
    f = native.ILU0(M)
    LU = sp.csr_matrix((f.lu, f.ci, f.rp), shape=M.shape).toarray()
    L = np.tril(LU, -1) + np.eye(80)
    U = np.triu(LU)
    b = np.random.default_rng(5).standard_normal(80)
    ref = sla.solve_triangular(U, sla.solve_triangular(L, b, lower=True, unit_diagonal=True))
    assert np.allclose(f.solve(b), ref, rtol=1e-12, atol=1e-13)


def test_levels_of_tridiagonal_are_sequential():
    n = 17
    T = sp.diags([-np.ones(n - 1), 4 * np.ones(n), -np.ones(n - 1)], [-1, 0, 1]).tocsr()
    assert native.levels(T, True)[0] == n
    assert native.levels(sp.eye(n, format="csr"), True)[0] == 1


# --------------------------------------------------------------- GMRES / CG --
def krylov_lsq_residuals(Aop, r0, k):
    """min_{y} ||r0 - Aop(V y)|| over span{r0, B r0, ...} built densely."""
    n = r0.size
    V = np.zeros((n, k))
    v = r0 / np.linalg.norm(r0)
    out = []
    for j in range(k):
        V[:, j] = v
        Q, _ = np.linalg.qr(V[:, :j + 1])
        W = np.column_stack([Aop(Q[:, i]) for i in range(j + 1)])
        y, *_ = np.linalg.lstsq(W, r0, rcond=None)
        out.append(np.linalg.norm(r0 - W @ y))
        v = Aop(v)
        v = v / np.linalg.norm(v)
    return np.array(out)


@pytest.mark.parametrize("side", ["left", "right"])
def test_gmres_estimates_are_minimal_residuals(side):
    A = rand_spd(120, density=0.05, seed=7, shift=0.05)
    pc = petsc.PCJacobi(A)
    b = np.random.default_rng(8).standard_normal(120)
    ksp = petsc.KSP(A, pc, "gmres", rtol=1e-12, atol=0, maxit=12, restart=50, pc_side=side)
    x = ksp.solve(b)
    if side == "right":
        ref = krylov_lsq_residuals(lambda v: A @ pc.apply(v), b, 12)
        assert np.isclose(ksp.history[-1], np.linalg.norm(b - A @ x), rtol=1e-8)
    else:
        r0 = pc.apply(b)
        ref = krylov_lsq_residuals(lambda v: pc.apply(A @ v), r0, 12)
        assert np.isclose(ksp.history[-1], np.linalg.norm(pc.apply(b - A @ x)), rtol=1e-8)
    assert np.allclose(ksp.history[1:], ref, rtol=1e-7)
    assert ksp.its == 12 and ksp.reason == petsc.DIVERGED_ITS


def test_gmres_hand_2x2_converges_in_two():
    A = sp.csr_matrix(np.array([[2.0, 1.0], [0.0, 3.0]]))
    b = np.array([0.0, 1.0])  # A b = [1, 3] is not parallel to b: two Krylov steps
    ksp = petsc.KSP(A, petsc.PCNone(), "gmres", rtol=1e-14, atol=1e-300, maxit=10, pc_side="right")
    x = ksp.solve(b)
    assert ksp.its == 2
    assert np.allclose(x, [-1.0 / 6.0, 1.0 / 3.0], rtol=1e-14)
    # an eigenvector right-hand side converges in one step (happy breakdown path not taken)
    ksp1 = petsc.KSP(A, petsc.PCNone(), "gmres", rtol=1e-14, atol=1e-300, maxit=10, pc_side="right")
    x1 = ksp1.solve(np.array([1.0, 1.0]))
    assert ksp1.its == 1 and np.allclose(x1, [1.0 / 3.0, 1.0 / 3.0], rtol=1e-14)


def test_gmres_restart_matches_fresh_cycles():
    A = rand_spd(80, density=0.08, seed=9, shift=0.02)
    b = np.random.default_rng(10).standard_normal(80)
    ksp = petsc.KSP(A, petsc.PCNone(), "gmres", rtol=1e-10, atol=0, maxit=400, restart=5, pc_side="right")
    x = ksp.solve(b)
    assert ksp.reason == petsc.CONVERGED_RTOL
    # restarted: the history restarts from the true residual at multiples of 5
    h = np.asarray(ksp.history)
    assert len(h) == ksp.its + 1 + (ksp.its - 1) // 5
    assert np.linalg.norm(b - A @ x) <= 1.01e-10 * np.linalg.norm(b)


def textbook_cg(A, b, M, maxit, rtol):
    x = np.zeros_like(b)
    r = b.copy()
    z = M(r)
    p = z.copy()
    rz = r @ z
    hist = [np.linalg.norm(r)]
    for _ in range(maxit):
        w = A @ p
        a = rz / (p @ w)
        x = x + a * p
        r = r - a * w
        hist.append(np.linalg.norm(r))
        if hist[-1] <= rtol * hist[0]:
            break
        z = M(r)
        rz_new = r @ z
        p = z + (rz_new / rz) * p
        rz = rz_new
    return x, np.array(hist)


def test_cg_matches_textbook():
    A = rand_spd(150, density=0.04, seed=11, shift=0.1)
    b = np.random.default_rng(12).standard_normal(150)
    pc = petsc.PCJacobi(A)
    ksp = petsc.KSP(A, pc, "cg", rtol=1e-8, atol=0, maxit=500, norm_type="unpreconditioned")
    x = ksp.solve(b)
    xr, hr = textbook_cg(A, b, pc.apply, 500, 1e-8)
    assert ksp.its == len(hr) - 1
    assert np.allclose(ksp.history, hr, rtol=1e-9)
    assert np.allclose(x, xr, rtol=1e-9, atol=1e-12)


def test_cg_indefinite_pc_stops_like_petsc():
    """cg.c: when (z, r) changes sign between iterations the PC is indefinite
    and KSPSolve_CG stops with KSP_DIVERGED_INDEFINITE_PC (-8) instead of
    running to max_it (ILU(0) of footing's undrained solid block does this).
    Against a textbook CG that records (z, r) per iteration."""
    A = rand_spd(60, density=0.1, seed=5, shift=0.5)
    d = np.ones(60)
    d[::3] = -0.2  # an indefinite diagonal PC

    class PCSigned:
        type = "signed"

        def apply(self, r):
            return d * r

    b = np.random.default_rng(6).standard_normal(60)
    ksp = petsc.KSP(A, PCSigned(), "cg", rtol=1e-12, atol=0, maxit=500, norm_type="unpreconditioned")
    ksp.solve(b)
    assert petsc.DIVERGED_INDEFINITE_PC == -8 and petsc.DIVERGED_INDEFINITE_MAT == -10  # petscksp.h
    # textbook CG: the first iteration whose beta = (z, r) has the other sign
    x, r = np.zeros(60), b.copy()
    z = d * r
    beta, p, k = z @ r, None, 0
    betas = [beta]
    while True:
        p = z.copy() if p is None else z + (beta / betas[-2]) * p
        w = A @ p
        a = beta / (p @ w)
        x, r = x + a * p, r - a * w
        z = d * r
        beta = z @ r
        betas.append(beta)
        k += 1
        if beta * betas[-2] < 0:
            break
    assert ksp.reason == petsc.DIVERGED_INDEFINITE_PC
    assert ksp.its == k + 1


def test_converged_default():
    c = petsc.ConvergedDefault(rtol=1e-2, atol=1e-5, dtol=10.0)
    assert c(0, 1.0) == 0
    assert c(1, 0.5) == 0
    assert c(2, 0.009) == petsc.CONVERGED_RTOL
    assert c(3, 1e-6) == petsc.CONVERGED_ATOL
    assert c(4, 11.0) == petsc.DIVERGED_DTOL
    assert c(5, float("nan")) == petsc.DIVERGED_NANORINF


def test_preonly():
    A = rand_spd(30, seed=13)
    ksp = petsc.KSP(A, petsc.PCLU(A), "preonly")
    b = np.ones(30)
    assert np.allclose(A @ ksp.solve(b), b)
    assert ksp.its == 1 and ksp.reason == petsc.CONVERGED_ITS


def test_side_norm_resolution():
    assert petsc.resolve_side_norm("gmres", None, None) == ("left", "preconditioned")
    assert petsc.resolve_side_norm("gmres", None, "unpreconditioned") == ("right", "unpreconditioned")
    assert petsc.resolve_side_norm("gmres", "right", None) == ("right", "unpreconditioned")
    with pytest.raises(ValueError):
        petsc.resolve_side_norm("gmres", "left", "unpreconditioned")


def test_bjacobi_block_sizes():
    assert petsc.bjacobi_block_sizes(10, 3) == [4, 3, 3]
    assert petsc.bjacobi_block_sizes(9, 3) == [3, 3, 3]
    M = rand_spd(40, seed=14)
    pc = petsc.PCBJacobi(M, 3, "ilu")
    x = np.random.default_rng(15).standard_normal(40)
    y = pc.apply(x)
    for lo, hi in zip(pc.bounds[:-1], pc.bounds[1:]):
        assert np.allclose(y[lo:hi], native.ILU0(M[lo:hi, lo:hi].tocsr()).solve(x[lo:hi]))


# ------------------------------------------------------------------ options --
def test_options_file_semantics():
    db = options.parse_options_lines([
        "-global_ksp_type gmres\n", "#-s_ksp_monitor\n", "-s_pc_type   lu\n",
        "-fp_ksp_gmres_modifiedgramschmidt\n", "   \n", "-p_ksp_rtol 1e-2 # trailing\n",
    ])
    assert db == {"global_ksp_type": "gmres", "s_pc_type": "lu", "fp_ksp_gmres_modifiedgramschmidt": None}


def test_repo_option_sets_parse():
    """The option sets shipped in options/ (exact, inexact-ilu, gpu-bjacobi)."""
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ex = options.parse_options_file(os.path.join(root, "options", "exact"))
    assert ex["global_ksp_type"] == "gmres" and ex["global_ksp_pc_side"] == "right"
    assert all(ex[p + "pc_type"] == "lu" for p in ("s_", "f_", "p_", "diff_", "fp_"))
    inex = options.parse_options_file(os.path.join(root, "options", "inexact-ilu"))
    assert inex["global_ksp_norm_type"] == "unpreconditioned" and inex["s_ksp_type"] == "cg"
    gb = options.parse_options_file(os.path.join(root, "options", "gpu-bjacobi"))
    assert gb["s_pc_type"] == "bjacobi" and int(gb["fp_pc_bjacobi_blocks"]) == 264


def test_local_fp_dofs():
    f, p = local_fp_dofs([1, 2, 5, 7, 8], [2, 7, 8], [1, 5])
    assert list(f) == [1, 3, 4] and list(p) == [0, 2]


# ----------------------------------------------------------------- block PC --
def _small_system(dim=2, N=5):
    spec = S.SynthSpec(dim, N)
    A, P, Pd = S.matrix(spec, 0), S.matrix(spec, 1), S.matrix(spec, 2)
    return spec, A, P, Pd


def test_block_pc_2way_exact_is_block_lower_solve():
    spec, A, P, Pd = _small_system()
    ns, nf, np_ = spec.sizes()
    is_s, is_f, is_p = S.field_major_index_sets(spec)
    is_fp = np.concatenate([is_f, is_p])
    db = {"s_ksp_type": "preonly", "s_pc_type": "lu", "fp_ksp_type": "preonly", "fp_pc_type": "lu"}
    pc = BP.BlockPC(P, Pd, (is_s, is_f, is_p, is_fp), (ns, nf, np_), False, db, "preonly", "lu")
    x = np.random.default_rng(16).standard_normal(spec.n)
    y = pc.apply(x)
    M = P.toarray()
    M[:ns, ns:] = 0.0  # block lower triangular [[K_s, 0], [P_fp,s, K_fp]]
    assert np.allclose(M @ y, x, rtol=1e-10, atol=1e-11)


def test_block_pc_3way_fs_and_diff_sweeps():
    spec, A, P, Pd = _small_system()
    ns, nf, np_ = spec.sizes()
    is_s, is_f, is_p = S.field_major_index_sets(spec)
    bcs = S.bcs_sub_pressure(spec)
    db = {k + "ksp_type": "preonly" for k in ("s_", "f_", "p_", "diff_")}
    db.update({k + "pc_type": "lu" for k in ("s_", "f_", "p_", "diff_")})
    pc = BP.BlockPC(P, Pd, (is_s, is_f, is_p, np.concatenate([is_f, is_p])), (ns, nf, np_), True, db, "preonly", "lu",
                    bcs_sub_pressure=bcs)
    x = np.random.default_rng(17).standard_normal(spec.n)
    y = pc.apply(x)
    # FS: block upper [[K_s, P_sf, P_sp], [0, K_f, P_fp], [0, 0, K_p]] y_FS = x
    U = np.triu(np.ones((3, 3)))
    off = [0, ns, ns + nf, spec.n]
    Mfs = P.toarray()
    for a in range(3):
        for b in range(3):
            if not U[a, b]:
                Mfs[off[a]:off[a + 1], off[b]:off[b + 1]] = 0.0
    y_fs = np.linalg.solve(Mfs, x)
    Mdf = Mfs.copy()
    Mdf[off[2]:, off[2]:] = Pd.toarray()[off[2]:, off[2]:]
    xd = x.copy()
    xd[off[2] + bcs] = 0.0
    y_df = np.linalg.solve(Mdf, xd)
    assert np.allclose(y, 1.0 * y_fs + 0.1 * y_df, rtol=1e-9, atol=1e-11)


def test_block_pc_rejects_bad_type():
    with pytest.raises(SystemExit, match="pc type must be one of"):
        BP.make_block_pc(None, None, None, None, {"pc type": "bogus"}, {}, [])


def test_fieldsplit_default_is_gmres_multiplicative():
    """Inexact inner PC without fp_ options: fp_ is GMRES + PCFIELDSPLIT with
    PETSc's defaults (MULTIPLICATIVE, split KSPs PREONLY + ILU), split 0 = p
    (Preconditioner.py:102-118)."""
    spec, A, P, Pd = _small_system()
    is_s, is_f, is_p = S.field_major_index_sets(spec)
    params = {"pc type": "diagonal", "inner ksp type": "cg", "inner pc type": "ilu", "inner accel order": 0,
              "solver type": "gmres", "solver atol": 1e-8, "solver rtol": 1e-6, "solver maxiter": 50}
    o = OracleSolver(A, P, Pd, is_s, is_f, is_p, params, {}, [])
    fs = o.block_pc.ksp_fp.pc
    assert o.block_pc.ksp_fp.type == "gmres" and fs.type == "fieldsplit" and fs.ftype == "multiplicative"
    assert np.array_equal(fs.is0, np.asarray(o.block_pc.is_p)) and fs.k0.type == "preonly"
    o.solve(S.rhs(spec))
    assert o.reason > 0


# ----------------------------------------------------------------- AAR -------
def test_aar_order0_is_richardson():
    A = rand_spd(50, seed=18, shift=2.0)
    pc = petsc.PCJacobi(A)
    b = np.random.default_rng(19).standard_normal(50)
    s = AA.AAR(0, 5, 1.0, 1.0, A, pc, atol=0, rtol=1e-6, maxiter=400)
    x = s.solve(b)
    xr = np.zeros(50)
    hist = [np.linalg.norm(b)]
    for _ in range(s.it):
        f = pc.apply(b - A @ xr)
        xr = xr + f
        hist.append(np.linalg.norm(f))
    assert np.allclose(x, xr, rtol=1e-12, atol=1e-14)
    assert np.allclose(s.history, hist, rtol=1e-12)


def test_aar_anderson_step_pairing_and_lstsq():
    """Trace the list bookkeeping of AAR.py:75-116 for order=3, p=2."""
    A = rand_spd(40, seed=20, shift=1.0)
    pc = petsc.PCJacobi(A)
    b = np.random.default_rng(21).standard_normal(40)
    s = AA.AAR(3, 2, 1.0, 1.0, A, pc, atol=0, rtol=0, maxiter=2)
    s.solve(b)
    # it=0 Richardson; it=1 Anderson with F0 = [df0, df1] (2 columns) and mk = 1
    x0 = np.zeros(40)
    f_prev = b.copy()
    f0 = pc.apply(b - A @ x0)
    df0 = f0 - f_prev
    x1 = x0 + f0
    dx0 = x1 - x0
    f1 = pc.apply(b - A @ x1)
    df1 = f1 - f0
    F = np.column_stack([df0, df1])
    alpha, *_ = np.linalg.lstsq(F, -f1, rcond=None)
    x2 = x1 + f1 + alpha[0] * (dx0 + df0)  # only the first mk = 1 coefficient, paired (X[0], F[0])
    s2 = AA.AAR(3, 2, 1.0, 1.0, A, pc, atol=0, rtol=0, maxiter=2)
    x = s2.solve(b)
    assert np.allclose(x, x2, rtol=1e-10, atol=1e-12)


def test_anderson_mixing_order0_identity():
    m = AA.AndersonAcceleration(0)
    g = np.arange(5.0)
    assert np.allclose(m.get_next_vector(g), g)


# -------------------------------------------------------------- synthetic ---
@pytest.mark.parametrize("dim,N", [(2, 3), (2, 7), (3, 2)])
def test_synthetic_structure(dim, N):
    spec = S.SynthSpec(dim, N)
    ns, nf, np_ = spec.sizes()
    q, v = 2 * N + 1, N + 1
    if dim == 3:
        assert (ns, nf, np_) == (3 * q ** 3, 3 * q ** 3, v ** 3)
    else:
        assert (ns, nf, np_) == (2 * q ** 2, 2 * q ** 2, v ** 2)
    for variant in (0, 1):
        M = S.matrix(spec, variant)
        assert abs(M - M.T).max() == 0.0
        d = M.diagonal()
        off = np.asarray(abs(M).sum(axis=1)).ravel() - d
        assert np.all(d > off)
        if M.shape[0] < 2000:
            assert np.linalg.eigvalsh(M.toarray()).min() > 0
    Pd = S.matrix(spec, 2)
    bc = S.bcs_sub_pressure(spec) + ns + nf
    R = Pd[bc].toarray()
    assert np.allclose(R.sum(axis=1), 1.0) and np.allclose(R[np.arange(len(bc)), bc], 1.0)


def test_synthetic_nnz_close_to_survey_2d_n32():
    spec = S.SynthSpec(2, 32)
    A = S.matrix(spec)
    assert spec.n == 17989
    assert abs(A.nnz / 927449 - 1) < 0.02  # SURVEY.md 8(a) dolfin-derived count


def numpy_enumeration(spec):
    """Independent numpy restatement of the synthetic pattern + values."""
    ns, nf, np_ = spec.sizes()
    n = (ns, nf, np_)
    off = (0, ns, ns + nf)
    blk = {(0, 0): 0, (0, 1): 1, (1, 0): 1, (0, 2): 2, (2, 0): 2, (1, 1): 3, (1, 2): 4, (2, 1): 4, (2, 2): 5}
    D = {b: spec.offsets(b) for b in range(6)}
    rows, cols = [], []
    for a in range(3):
        i = np.arange(n[a], dtype=np.int64)
        for b in range(3):
            d = D[blk[(a, b)]].astype(np.int64)
            if a <= b:
                ctr = i if a == b else (i * n[b]) // n[a]
                J = ctr[:, None] + d[None, :]
                ok = (J >= 0) & (J < n[b])
                rr, cc = np.nonzero(ok)
                rows.append(off[a] + i[rr])
                cols.append(off[b] + J[rr, cc])
            else:
                j = np.arange(n[b], dtype=np.int64)
                ctr = (j * n[a]) // n[b]
                I = ctr[:, None] + d[None, :]
                ok = (I >= 0) & (I < n[a])
                rr, cc = np.nonzero(ok)
                rows.append(off[a] + I[rr, cc])
                cols.append(off[b] + j[rr])
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    lo, hi = np.minimum(r, c), np.maximum(r, c)
    u = (S._hash3(np.uint64(spec.seed) ^ np.uint64(0x5A1BE5), lo.astype(np.uint64), hi.astype(np.uint64))
         >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    fa = np.searchsorted(np.array(off[1:]), r, side="right")
    fb = np.searchsorted(np.array(off[1:]), c, side="right")
    v = np.where(fa == fb, -u, -(0.1 * u))
    v[r == c] = 0.0
    M = sp.csr_matrix((v, (r, c)), shape=(spec.n, spec.n))
    M.sort_indices()
    return M


@pytest.mark.parametrize("dim,N", [(2, 4), (3, 2)])
def test_synthetic_c_matches_numpy_enumeration(dim, N):
    spec = S.SynthSpec(dim, N)
    M = S.matrix(spec, 0)
    R = numpy_enumeration(spec)
    assert np.array_equal(M.indptr, R.indptr) and np.array_equal(M.indices, R.indices)
    off = M.copy()
    off.setdiag(0.0)
    assert np.array_equal(off.toarray(), R.toarray())


# ---------------------------------------------------------- fieldsplit ----
def _fp_block(N=6):
    from oracle import synthetic as S
    spec = S.SynthSpec(2, N)
    P = S.matrix(spec, 1)
    ns, nf, np_ = spec.sizes()
    K = P[ns:, ns:].tocsr()
    return K, np.arange(nf, nf + np_), np.arange(nf)


def test_fieldsplit_schur_full_exact_inverts_block():
    """Schur FULL with exact split-0 solves and a converged Schur KSP (implicit
    S = A11 - A10 A00^-1 A01, preconditioned by LU(selfp)) is K^-1."""
    from oracle.fieldsplit import PCFieldSplit
    K, is_p, is_f = _fp_block()
    db = {"fp_pc_fieldsplit_type": "schur", "fp_pc_fieldsplit_schur_fact_type": "full",
          "fp_pc_fieldsplit_schur_precondition": "selfp",
          "fp_fieldsplit_0_ksp_type": "preonly", "fp_fieldsplit_0_pc_type": "lu",
          "fp_fieldsplit_1_ksp_type": "gmres", "fp_fieldsplit_1_ksp_rtol": "1e-13",
          "fp_fieldsplit_1_pc_type": "lu"}
    pc = PCFieldSplit(K, is_p, is_f, db, "fp_")
    x = np.random.default_rng(3).standard_normal(K.shape[0])
    y = pc.apply(x)
    assert np.linalg.norm(K @ y - x) <= 1e-10 * np.linalg.norm(x)


def test_fieldsplit_selfp_definition():
    """SELFP = A11 - A10 diag(A00)^-1 A01 (dense check)."""
    from oracle.fieldsplit import PCFieldSplit
    K, is_p, is_f = _fp_block(4)
    pc = PCFieldSplit(K, is_p, is_f, {"fp_pc_fieldsplit_type": "schur",
                                      "fp_pc_fieldsplit_schur_precondition": "selfp"}, "fp_")
    Kd = K.toarray()
    A00, A01 = Kd[np.ix_(is_p, is_p)], Kd[np.ix_(is_p, is_f)]
    A10, A11 = Kd[np.ix_(is_f, is_p)], Kd[np.ix_(is_f, is_f)]
    ref = A11 - A10 @ np.diag(1.0 / np.diag(A00)) @ A01
    assert np.allclose(pc.Sp.toarray(), ref, rtol=1e-14, atol=1e-14)


@pytest.mark.parametrize("ftype,fact", [("additive", None), ("multiplicative", None), ("schur", "diag"),
                                        ("schur", "lower"), ("schur", "upper")])
def test_fieldsplit_block_factorizations(ftype, fact):
    """With exact sub-solves (LU on A00, LU on A11 or on S via selfp when S is
    replaced by its LU), each variant is the stated block-triangular solve."""
    from oracle.fieldsplit import PCFieldSplit
    K, is_p, is_f = _fp_block(4)
    db = {"fp_pc_fieldsplit_type": ftype, "fp_fieldsplit_0_pc_type": "lu", "fp_fieldsplit_1_pc_type": "lu",
          "fp_fieldsplit_1_ksp_type": "preonly"}
    if fact:
        db["fp_pc_fieldsplit_schur_fact_type"] = fact
        db["fp_pc_fieldsplit_schur_precondition"] = "a11"
    pc = PCFieldSplit(K, is_p, is_f, db, "fp_")
    Kd = K.toarray()
    A00, A01 = Kd[np.ix_(is_p, is_p)], Kd[np.ix_(is_p, is_f)]
    A10, A11 = Kd[np.ix_(is_f, is_p)], Kd[np.ix_(is_f, is_f)]
    x = np.random.default_rng(4).standard_normal(K.shape[0])
    x0, x1 = x[is_p], x[is_f]
    inv = np.linalg.solve
    if ftype == "additive":
        y0, y1 = inv(A00, x0), inv(A11, x1)
    elif ftype == "multiplicative" or fact == "lower":
        y0 = inv(A00, x0)
        y1 = inv(A11, x1 - A10 @ y0)
    elif fact == "diag":
        y0, y1 = inv(A00, x0), -inv(A11, x1)
    else:  # upper
        y1 = inv(A11, x1)
        y0 = inv(A00, x0 - A01 @ y1)
    y = pc.apply(x)
    assert np.allclose(y[is_p], y0, rtol=1e-10, atol=1e-12)
    assert np.allclose(y[is_f], y1, rtol=1e-10, atol=1e-12)


# ------------------------------------------------- C/OpenMP CPU baseline ----
@pytest.mark.parametrize("threads", [1, 4])
def test_cpu_baseline_solver_matches_oracle(threads):
    """oracle/csrc/cpu_solver.c (bench.py's cpu_baseline) == the Python oracle
    on bench's configuration: same iteration count and reason, history to
    rounding (its inner products are OpenMP reductions)."""
    spec = S.SynthSpec(2, 12)
    A, P = S.matrix(spec, 0), S.matrix(spec, 1)
    ns = spec.sizes()[0]
    is_s, is_f, is_p = S.field_major_index_sets(spec)
    params = {"solver type": "gmres", "solver atol": 1e-8, "solver rtol": 1e-6, "solver maxiter": 100,
              "pc type": "diagonal", "inner ksp type": "preonly", "inner pc type": "bjacobi",
              "inner accel order": 0}
    db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "s_ksp_type": "preonly",
          "s_pc_type": "bjacobi", "s_pc_bjacobi_blocks": "5", "fp_ksp_type": "preonly",
          "fp_pc_type": "bjacobi", "fp_pc_bjacobi_blocks": "3"}
    o = OracleSolver(A, P, None, is_s, is_f, is_p, params, db, [])
    b = S.rhs(spec)
    xo = o.solve(b)
    x, its, reason, hist, _, _ = native.cpu_gmres_2way(A, P, ns, 5, 3, b, nthreads=threads)
    assert its == o.its and reason == o.reason
    assert np.allclose(hist, o.history, rtol=1e-10, atol=0)
    assert np.allclose(x, xo, rtol=1e-9, atol=1e-12)
