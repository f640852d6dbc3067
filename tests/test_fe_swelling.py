"""The P2-P2-P1 swelling assembler (lib/fe_swelling.py): sizes and sparsity
against SURVEY.md 8(a)'s dolfin-pattern formulas, element identities, the
block structure of lib/Assembler.py's forms, dolfin's Dirichlet rows, and the
oracle solving the assembled systems (CPU; the GPU comparison is
tests/test_gpu_fe.py)."""
import numpy as np
import pytest
import scipy.sparse.linalg as spl

from lib import fe_swelling as F


def _n(dim, N):
    return 6 * (2 * N + 1) ** 3 + (N + 1) ** 3 if dim == 3 else 4 * (2 * N + 1) ** 2 + (N + 1) ** 2


@pytest.mark.parametrize("dim,N", [(2, 32), (2, 5), (3, 2), (3, 4)])
def test_sizes_and_nnz_match_dolfin_pattern(dim, N):
    """n = 6(2N+1)^3 + (N+1)^3 (3-D), 4(2N+1)^2 + (N+1)^2 (2-D);
    nnz_3D(N) = 9075N^3 + 5673N^2 + 1053N + 49; 2-D N=32: 927,449."""
    s = F.assemble_swelling(dim, N, "diagonal 3-way")
    assert s.A.shape == (_n(dim, N),) * 2
    assert s.dims == ((dim * (2 * N + 1) ** dim,) * 2 + ((N + 1) ** dim,))
    if dim == 3:
        assert s.A.nnz == 9075 * N ** 3 + 5673 * N ** 2 + 1053 * N + 49
    elif N == 32:
        assert s.A.nnz == 927449
    for M in (s.P, s.P_diff):  # one pattern for A, P, P_diff (explicit zeros kept)
        assert np.array_equal(M.indptr, s.A.indptr) and np.array_equal(M.indices, s.A.indices)
    pat = s.A.copy()
    pat.data[:] = 1
    assert abs(pat - pat.T).nnz == 0
    assert np.array_equal(np.sort(np.concatenate([s.is_s, s.is_f, s.is_p])), np.arange(s.A.shape[0]))


@pytest.mark.parametrize("dim", [2, 3])
def test_element_identities(dim):
    """Exact integrals of the elementary forms on linear fields: P2/P1 mass
    sums to the volume, eps:eps of (x,0) = 1 and of (y,0) = 1/2 per unit
    volume, rigid rotations have zero strain energy, div(x,0) = 1 against
    every P1 test function, grad 1 = 0, |grad x|^2 = 1."""
    N = 3
    h = F.SIDE_LENGTH / N
    coords, cells, pairs, cn, node2x, nv = F._p2_nodes(dim, N)
    M2, G, C, Mp, Kp = F._element_blocks(dim, coords[cells] * h)
    Mv, E, Dd, Bt = F._vector_blocks(dim, M2, G, C)
    X = node2x * h / 2
    vol = F.SIDE_LENGTH ** dim
    z = np.zeros(len(X))

    def energy(K, u):
        uc = u[cn].reshape(cn.shape[0], -1)
        return np.einsum("ci,cij,cj->", uc, K, uc)

    u1 = np.stack([X[:, 0]] + [z] * (dim - 1), 1)
    u2 = np.stack([X[:, 1]] + [z] * (dim - 1), 1)
    rot = np.stack([-X[:, 1], X[:, 0]] + [z] * (dim - 2), 1)
    assert M2.sum() == pytest.approx(vol, rel=1e-13) and Mp.sum() == pytest.approx(vol, rel=1e-13)
    assert energy(E, u1) == pytest.approx(vol, rel=1e-12)
    assert energy(E, u2) == pytest.approx(vol / 2, rel=1e-12)
    assert abs(energy(E, rot)) <= 1e-12 * vol
    assert energy(Dd, u1) == pytest.approx(vol, rel=1e-12)
    bq = np.einsum("cie,ci->ce", Bt, u1[cn].reshape(cn.shape[0], -1))
    assert np.max(np.abs(bq - Mp.sum(2))) <= 1e-13 * np.max(Mp.sum(2))
    assert np.max(np.abs(Kp.sum(2))) <= 1e-12 * np.max(np.abs(Kp))
    px = X[:nv, 0][cells]
    assert np.einsum("ci,cij,cj->", px, Kp, px) == pytest.approx(vol, rel=1e-12)


def _block(M, r, c):
    return M[r][:, c]


def test_form_structure_base_matrix():
    """lib/Assembler.py:78-97, away from Dirichlet rows: A_sp = -phis B and
    A_ps = (phis/dt) B^T give A_sp = -dt A_ps^T; A_fp = -phi0 B and
    A_pf = phi0 B^T give A_fp = -A_pf^T; A_sf = -phi0^2/kf M and
    A_fs = -phi0^2/(kf dt) M give A_sf = dt A_fs^T; A_ss is symmetric."""
    s = F.assemble_swelling(2, 6, "diagonal")
    prm = F.SWELLING_2D
    dt, phi0 = prm["dt"], prm["phi0"]
    phis = 1 - phi0
    bc = np.nonzero(np.isclose(s.A.diagonal(), 1.0) & (np.diff(s.A.indptr) > 0) &
                    (abs(s.A).sum(1).A.ravel() == 1.0))[0]
    keep_s = np.setdiff1d(s.is_s, bc)
    keep_f = np.setdiff1d(s.is_f, bc)
    A = s.A.tocsr()
    sp_ = _block(A, keep_s, s.is_p).toarray()
    ps_ = _block(A, s.is_p, keep_s).toarray()
    assert np.allclose(sp_, -dt * ps_.T, rtol=1e-12, atol=1e-12 * np.abs(sp_).max())
    fp_ = _block(A, keep_f, s.is_p).toarray()
    pf_ = _block(A, s.is_p, keep_f).toarray()
    assert np.allclose(fp_, -pf_.T, rtol=1e-12, atol=1e-12 * np.abs(fp_).max())
    ss = _block(A, keep_s, keep_s).toarray()
    assert np.allclose(ss, ss.T, rtol=1e-12, atol=1e-12 * np.abs(ss).max())
    sf = _block(A, keep_s, keep_f).toarray()
    fs = _block(A, keep_f, keep_s).toarray()
    assert np.allclose(sf, dt * fs.T, rtol=1e-12, atol=1e-12 * np.abs(sf).max())
    # "diagonal" P drops the f->s and p->s couplings (Assembler.py:149-168)
    assert _block(s.P, s.is_f, s.is_s).count_nonzero() == 0
    assert _block(s.P, s.is_p, s.is_s).count_nonzero() == 0


def test_dirichlet_rows_and_pressure_bcs():
    """dolfin DirichletBC.apply: unit rows in A and P at the solid / fluid bc
    dofs, zero b there; pressure bcs only in P_diff; bcs_sub_pressure indexes
    the p sub-vector (lib/Poromechanics.py:40-55,72-83)."""
    N = 4
    s = F.assemble_swelling(2, N, "diagonal 3-way")
    unit = []
    for M in (s.A, s.P, s.P_diff):
        rows = [r for r in range(M.shape[0]) if np.count_nonzero(M.getrow(r).data) == 1 and M[r, r] == 1.0]
        unit.append(set(rows))
    assert unit[0] == unit[1]
    bc = sorted(unit[0])
    assert np.all(s.b[bc] == 0.0)
    # swelling.py:93-98: u_s,x on LEFT (2N+1 nodes), u_s,y on BOTTOM, v_f on TOP and BOTTOM (2 x 2(2N+1) - shared: none)
    assert len(bc) == (2 * N + 1) * 2 + 2 * 2 * (2 * N + 1)
    p_bc = unit[2] - unit[0]
    # LEFT, TOP, RIGHT pressure vertices: 3(N+1) - 2 corners
    assert len(p_bc) == 3 * (N + 1) - 2 == len(s.bcs_sub_pressure)
    assert set(s.is_p[s.bcs_sub_pressure]) == p_bc


def test_orderings_are_one_system():
    """field-major and interleaved numberings: the same operator after
    restriction to the index sets (same node order inside each field)."""
    a = F.assemble_swelling(2, 5, "diagonal 3-way", ordering="field-major")
    b = F.assemble_swelling(2, 5, "diagonal 3-way", ordering="interleaved")
    ia = np.concatenate([a.is_s, a.is_f, a.is_p])
    ib = np.concatenate([b.is_s, b.is_f, b.is_p])
    assert not np.array_equal(a.is_p, b.is_p)
    for Ma, Mb in ((a.A, b.A), (a.P, b.P), (a.P_diff, b.P_diff)):
        d = (Ma[ia][:, ia] - Mb[ib][:, ib]).toarray()
        assert np.max(np.abs(d)) <= 1e-14 * abs(Ma).max()
    assert np.allclose(a.b[ia], b.b[ib], rtol=0, atol=1e-15 * np.abs(a.b).max())
    assert np.array_equal(a.bcs_sub_pressure, b.bcs_sub_pressure)


def test_surface_load_total():
    """Total surface load: the solid y-components carry c_s n_y over TOP (no
    u_s,y Dirichlet dof on TOP); the fluid x-components carry c_f n_x = -c_f
    over LEFT, less the two corner nodes that the v_f Dirichlet rows (TOP,
    BOTTOM) zero, h/6 each (swelling.py:21-22,36-41,93-98)."""
    N = 4
    s = F.assemble_swelling(2, N, "diagonal")
    t = F.SWELLING_2D["dt"]
    cs = -1e3 * 0.9 * (1 - np.exp(-t ** 2 / 0.25))
    cf = -1e3 * 0.1 * (1 - np.exp(-t ** 2 / 0.25))
    sy = s.is_s[1::2]
    assert s.b[sy].sum() == pytest.approx(cs * F.SIDE_LENGTH, rel=1e-12)
    fx = s.is_f[0::2]
    assert s.b[fx].sum() == pytest.approx(-cf * (F.SIDE_LENGTH - 2 * F.SIDE_LENGTH / N / 6), rel=1e-12)


BASE = {"solver type": "gmres", "solver atol": 1e-8, "solver rtol": 1e-6, "solver maxiter": 300,
        "pc type": "diagonal", "inner ksp type": "preonly", "inner pc type": "lu", "inner rtol": 1e-6,
        "inner atol": 0, "inner maxiter": 1000, "inner monitor": False, "solver monitor": False,
        "inner accel order": 0, "AAR order": 10, "AAR p": 5, "AAR omega": 1, "AAR beta": 1}


def _db(inner):
    d = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right"}
    for p in ("s_", "f_", "p_", "diff_", "fp_"):
        d[p + "ksp_type"] = "preonly"
        d[p + "pc_type"] = inner
    return d


@pytest.mark.parametrize("dim,N,pc,inner,its", [(2, 8, "diagonal", "lu", 8), (2, 8, "diagonal", "ilu", 36),
                                                (2, 8, "diagonal 3-way", "lu", 14), (3, 3, "diagonal", "lu", 7)])
def test_oracle_solves_assembled_system(dim, N, pc, inner, its):
    """The oracle's block-preconditioned GMRES on the assembled systems: the
    reference's default "diagonal" PC with exact blocks converges in a handful
    of iterations, and the solution agrees with a direct solve of A."""
    from oracle.solver import OracleSolver
    s = F.assemble_swelling(dim, N, pc)
    o = OracleSolver(s.A, s.P, s.P_diff, s.is_s, s.is_f, s.is_p, dict(BASE, **{"pc type": pc}), _db(inner),
                     s.bcs_sub_pressure)
    x = o.solve(s.b)
    assert o.reason > 0 and o.its == its
    xd = spl.spsolve(s.A.tocsc(), s.b)
    r = np.linalg.norm(s.A @ x - s.b)
    assert r <= max(1e-6 * np.linalg.norm(s.b), 1e-8) * 1.0001
    assert np.linalg.norm(x - xd) <= 0.1 * np.linalg.norm(xd)


def _fe_golden():
    import glob
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fe")
    return sorted(glob.glob(os.path.join(here, "*.npz")))


@pytest.mark.parametrize("path", _fe_golden(), ids=lambda p: p.rsplit("/", 1)[-1][:-4])
def test_fe_golden_fixtures(path):
    """tests/golden/fe (tests/golden/make_golden_fe.py): the assembler's matrix
    checksums and the oracle's solve on the assembled system are reproduced."""
    import json
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_golden_fe as G
    z = np.load(path, allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    name = os.path.basename(path)[:-4]
    s, params, db, o, x = G.run_case(name)
    assert np.allclose(G.checksums(s), z["checksums"], rtol=1e-13, atol=0)
    assert o.its == int(z["its"]) and o.reason == int(z["reason"])
    assert np.allclose(o.history, z["history"], rtol=1e-9, atol=0)
    assert np.allclose(x, z["x"], rtol=1e-8, atol=1e-12 * np.abs(z["x"]).max())
    assert meta["pc"] == params["pc type"]
