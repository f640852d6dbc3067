"""CPU tests of the classical-AMG specification behind -pc_type hypre
(oracle/boomeramg.py) and of libpls's host setup of it.

hypre is absent from this image and from the reference tree, so nothing here
is pinned against hypre's own numbers ("parity unpinned"):
* known-answer tests of the strength rule and the Ruge-Stueben first pass on
  hand-checked matrices;
* properties of the interpolations (extended+i and multipass reproduce the
  constant on zero-row-sum rows; P_max truncation keeps <= P_max entries and
  the row sums);
* convergence of PCG with one V-cycle per step (2-D Laplacian, 3-D FE
  elasticity block);
* libpls's host setup (pls_boomeramg_host_level, no device) equal to the
  oracle bit for bit -- C/F splitting, every P value, the coarsest operator --
  on the 2-D Laplacian, an anisotropic operator, the synthetic system's solid
  block and the assembled swelling blocks, with the reference's
  petsc-options-inexact settings and with PETSc's defaults.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import synthetic as S
from oracle.boomeramg import (C, F, PCBoomerAMG, coarsen, ext_i_interp, multipass_interp, rs_first_pass,
                              strength, truncate)

INEXACT = {"x_pc_hypre_boomeramg_P_max": "4", "x_pc_hypre_boomeramg_agg_nl": "1",
           "x_pc_hypre_boomeramg_agg_num_paths": "2", "x_pc_hypre_boomeramg_coarsen_type": "HMIS",
           "x_pc_hypre_boomeramg_interp_type": "ext+i", "x_pc_hypre_boomeramg_no_CF": "true",
           "x_pc_hypre_boomeramg_grid_sweeps_all": "1"}


def lap1(n):
    return sp.diags([-1.0, 2.0, -1.0], [-1, 0, 1], shape=(n, n)).tocsr()


def lap2(n, eps=1.0):
    I, T = sp.eye(n), lap1(n)
    return (sp.kron(I, T) + eps * sp.kron(T, I)).tocsr()


def neumann2(n):
    """2-D Laplacian with zero row sums everywhere (graph Laplacian of the grid)."""
    A = lap2(n).tolil()
    A.setdiag(0.0)
    A = A.tocsr()
    return (A - sp.diags(np.asarray(A.sum(axis=1)).ravel())).tocsr()


def pcg(A, b, M, rtol=1e-8, maxit=200):
    x = np.zeros_like(b)
    r = b.copy()
    z = M(r)
    p = z.copy()
    rz = r @ z
    for k in range(maxit):
        Ap = A @ p
        a = rz / (p @ Ap)
        x += a * p
        r -= a * Ap
        if np.linalg.norm(r) < rtol * np.linalg.norm(b):
            return k + 1
        z = M(r)
        rzn = r @ z
        p = z + rzn / rz * p
        rz = rzn
    return maxit


def test_strength_rule_kat():
    # row 0: d > 0, min off-diagonal -4: strong iff a < 0.25 * -4 = -1 -> col 1 (-4), not col 2 (-1), not col 3 (+2)
    # row 1: d < 0 (sign flipped rule): max off-diagonal 3: strong iff a > 0.75 -> col 0 (3), col 2 (1)
    # row 2: Dirichlet-like row (row sum == diagonal): no strong dependencies (max_row_sum 0.9)
    # row 3: only positive off-diagonals: nothing strong
    A = sp.csr_matrix(np.array([[10.0, -4.0, -1.0, 2.0],
                                [3.0, -8.0, 1.0, 0.5],
                                [0.0, 0.0, 5.0, 0.0],
                                [1.0, 0.0, 0.0, 4.0]]))
    Sl = strength(A, 0.25, 0.9)
    assert [s.tolist() for s in Sl] == [[1], [0, 2], [], []]
    # max_row_sum 1.0 disables the row-sum test; row 2 then has no off-diagonals anyway
    assert strength(A, 0.25, 1.0)[2].tolist() == []


def test_rs_first_pass_chain_kat():
    # 1-D Laplacian, 7 points: lambda = 1,2,2,2,2,2,1 -> 1 is C (largest, smallest index), 0, 2 F,
    # lambda_3 += 1 -> 3 C, 4 F, lambda_5 += 1 -> 5 C, 6 F
    cf = rs_first_pass(strength(lap1(7)), 7)
    assert cf.tolist() == [F, C, F, C, F, C, F]


def test_aggressive_coarsening_chain():
    # C1 = {1, 3, 5, 7, 9}; on C1 every pair at distance 2 is joined by exactly one
    # path of length 2, so agg_num_paths 1 coarsens again (every other C1 point)
    A = lap1(11)
    Sl = strength(A)
    cf1 = coarsen(Sl, 11, False, 1)
    assert np.flatnonzero(cf1 == C).tolist() == [1, 3, 5, 7, 9]
    cf = coarsen(Sl, 11, True, 1)
    assert np.flatnonzero(cf == C).tolist() == [3, 7]
    # num_paths 2: no pair of C1 points has 2 paths: S2 empty, nothing stays C
    assert np.flatnonzero(coarsen(Sl, 11, True, 2) == C).tolist() == []


@pytest.mark.parametrize("interp", ["ext+i", "multipass"])
def test_interpolation_reproduces_constants(interp):
    A = neumann2(12)
    n = A.shape[0]
    Sl = strength(A)
    cf = coarsen(Sl, n, interp == "multipass", 1)
    P = ext_i_interp(A, Sl, cf) if interp == "ext+i" else multipass_interp(A, Sl, cf)
    assert P.shape == (n, int((cf == C).sum()))
    one = P @ np.ones(P.shape[1])
    reached = np.diff(P.indptr) > 0
    assert reached.sum() > 0.9 * n
    assert np.allclose(one[reached], 1.0, rtol=0, atol=1e-13)
    # C points inject
    cidx = np.cumsum(cf == C) - 1
    for i in np.flatnonzero(cf == C)[:20]:
        row = P.getrow(i)
        assert row.indices.tolist() == [cidx[i]] and row.data.tolist() == [1.0]


def test_truncation_keeps_pmax_and_row_sums():
    A = lap2(14, eps=0.3)
    n = A.shape[0]
    Sl = strength(A)
    cf = coarsen(Sl, n, False, 1)
    P = ext_i_interp(A, Sl, cf)
    assert np.diff(P.indptr).max() > 2
    Pt = truncate(P, 2)
    assert np.diff(Pt.indptr).max() <= 2
    assert np.allclose(Pt @ np.ones(Pt.shape[1]), P @ np.ones(P.shape[1]), rtol=1e-14, atol=1e-15)
    for i in range(n):  # the kept entries are the 2 largest in magnitude
        full = np.sort(np.abs(P.getrow(i).data))[::-1]
        if full.size > 2:
            kept = P.getrow(i).data[np.isin(P.getrow(i).indices, Pt.getrow(i).indices)]
            assert Pt.getrow(i).nnz == 2 and np.abs(kept).min() >= full[1]


@pytest.mark.parametrize("db", [{}, INEXACT], ids=["defaults", "inexact"])
def test_vcycle_pcg_convergence_lap2(db):
    A = lap2(40)
    pc = PCBoomerAMG(A, db, "x_")
    assert len(pc.levels) >= 3
    b = np.random.default_rng(0).standard_normal(A.shape[0])
    assert pcg(A, b, pc.apply) <= 12


def test_vcycle_is_symmetric_no_cf():
    """Symmetric GS pre/post smoothing + Galerkin coarse operators: a symmetric operator."""
    A = lap2(16)
    pc = PCBoomerAMG(A, INEXACT, "x_")
    rng = np.random.default_rng(1)
    u, v = rng.standard_normal((2, A.shape[0]))
    assert abs(u @ pc.apply(v) - v @ pc.apply(u)) <= 1e-12 * np.linalg.norm(u) * np.linalg.norm(v)


def test_options_refused():
    with pytest.raises(NotImplementedError):
        PCBoomerAMG(lap2(5), {"x_pc_hypre_boomeramg_coarsen_type": "Falgout"}, "x_")


# ---------------------------------------------------- libpls host setup ----
def _blocks():
    out = [("lap2", lap2(30)), ("aniso", lap2(24, eps=0.01))]
    spec = S.SynthSpec(3, 4)
    A = S.matrix(spec)
    ns = spec.sizes()[0]
    out.append(("synth3d4_s", A[:ns, :ns].tocsr()))
    from lib.fe_swelling import assemble_swelling
    s = assemble_swelling(3, 3, "diagonal")
    B = s.A.tocsr()[s.is_s][:, s.is_s].tocsr()
    B.sort_indices()
    out.append(("fe3d3_s", B))
    return out


@pytest.mark.parametrize("db", [{}, INEXACT, dict(INEXACT, **{"pls.hypre_coarsen_chunks": "7"}),
                                dict(INEXACT, **{"pls.hypre_relax_min_rows": "64", "pls.hypre_coarsen_min_rows": "200",
                                                 "pls.hypre_coarsen_chunks": "0"})],
                         ids=["defaults", "inexact", "inexact-7-partitions", "inexact-chunked"])
def test_libpls_host_setup_bitwise(db):
    from lib.handle import boomeramg_host_level
    for name, A in _blocks():
        A = A.tocsr()
        A.sort_indices()
        pc = PCBoomerAMG(A, db, "x_")
        for l, L in enumerate(pc.levels):
            nl, n, nc, cf, P = boomeramg_host_level(A, db, "x_", l)
            assert nl == len(pc.levels) + 1, name
            assert np.array_equal(cf, L["cf"].astype(np.int8)), (name, l)
            Po = L["P"]
            assert np.array_equal(P.indptr, Po.indptr) and np.array_equal(P.indices, Po.indices), (name, l)
            assert np.array_equal(P.data, Po.data), (name, l)
        nl, n, nc, cf, Ac = boomeramg_host_level(A, db, "x_", len(pc.levels))
        Co = pc.coarse.tocsr()
        assert np.array_equal(Ac.indptr, Co.indptr) and np.array_equal(Ac.data, Co.data), name


# ------------------------------------------- hybrid Gauss-Seidel (K chunks) ----
@pytest.mark.parametrize("K", [1, 3, 7, 64, 1000])
@pytest.mark.parametrize("points", [None, "C", "F"])
def test_hybrid_sgs_matrix_form_equals_hypre_loop(K, points):
    """The spec's matrix form u_I += M^-1 (b - A u)_I, M = (D+L) D^-1 (D+U) of
    the chunk-block-diagonal part, equals hypre's relax type 6 with K threads
    row by row (par_relax.c: chunk rows read new values, the rest the values
    before the sweep), on a nonsymmetric matrix, nonzero start, C/F subsets."""
    from oracle.boomeramg import _sgs_factors, chunk_ids, hybrid_sgs_literal
    import scipy.sparse.linalg as spla
    rng = np.random.default_rng(K)
    A = (lap2(9, eps=0.4) + sp.random(81, 81, density=0.03, random_state=1)).tocsr()
    A.sort_indices()
    n = A.shape[0]
    b, u = rng.standard_normal((2, n))
    mask = None if points is None else (rng.random(n) < 0.4) ^ (points == "F")
    idx = None if mask is None else np.flatnonzero(mask)
    ref = hybrid_sgs_literal(A, b, u, K, mask)
    lo, up, us = _sgs_factors(A, chunk_ids(n, K), idx)
    r = (b - A @ u) if idx is None else (b - A @ u)[idx]
    d1 = spla.spsolve_triangular(lo, r, lower=True)
    d = d1 + spla.spsolve_triangular(up, -(us @ d1), lower=False)
    got = u.copy()
    if idx is None:
        got += d
    else:
        got[idx] += d
    assert np.max(np.abs(got - ref)) <= 1e-13 * np.max(np.abs(ref))


def test_chunk_partition_is_hypres():
    from oracle.boomeramg import chunk_ids
    c = chunk_ids(10, 4)  # size 2, rest 2: chunks of 3, 3, 2, 2
    assert c.tolist() == [0, 0, 0, 1, 1, 1, 2, 2, 3, 3]
    assert chunk_ids(3, 256).tolist() == [0, 1, 2]  # Jacobi when rows < K
    from oracle.boomeramg import level_chunks
    assert level_chunks(5_000_000, 256, 1024) == 256 and level_chunks(10_000, 256, 1024) == 9
    assert level_chunks(500, 256, 1024) == 1 and level_chunks(500, 256, 0) == 256


@pytest.mark.parametrize("K", [1, 8, 256])
def test_hybrid_vcycle_pcg_converges(K):
    A = lap2(40)
    pc = PCBoomerAMG(A, dict(INEXACT, **{"pls.hypre_relax_chunks": str(K), "pls.hypre_relax_min_rows": "0"}), "x_")
    b = np.random.default_rng(0).standard_normal(A.shape[0])
    assert pcg(A, b, pc.apply) <= 14


def test_partitioned_first_pass_is_per_partition():
    """HMIS's first pass inside each partition: the C/F splitting of a
    partitioned level equals the splittings of its partitions' own blocks."""
    from oracle.boomeramg import chunk_ids, rs_first_pass, rs_partitioned
    A = lap2(20)
    n = A.shape[0]
    S = strength(A)
    part = chunk_ids(n, 3)
    cf = rs_partitioned(S, n, part)
    for k in range(3):
        idx = np.flatnonzero(part == k)
        a, b = idx[0], idx[-1] + 1
        Sl = [row[(row >= a) & (row < b)] - a for row in S[a:b]]
        assert np.array_equal(cf[a:b], rs_first_pass(Sl, b - a))
    assert not np.array_equal(cf, rs_first_pass(S, n))  # the partition boundary changes the splitting


def test_hypre_rand_is_the_minimal_standard_generator():
    """hypre_Rand (Park-Miller, a = 16807, m = 2^31 - 1): the generator's
    published check values from seed 1 (16807, 282475249, 1622650073; the
    10,000th value 1043618065)."""
    from oracle.boomeramg import hypre_rand
    m = 2147483647
    v = hypre_rand(1, 10000) * m
    assert np.round(v[:3]).astype(np.int64).tolist() == [16807, 282475249, 1622650073]
    assert int(round(v[-1])) == 1043618065


@pytest.mark.parametrize("K", [1, 3, 8])
def test_pmis_stage_properties(K):
    """HMIS's PMIS stage over the per-partition first pass (lap2 and an
    anisotropic operator, K partitions): points without a strong dependency
    on another partition keep their first-pass decision (K = 1: the first
    pass itself); the boundary points PMIS makes C form an independent set of
    S; every boundary F point strongly depends on a C point or has no point
    depending on it."""
    from oracle.boomeramg import chunk_ids, pmis_stage, rs_partitioned, transpose_lists
    for A in (lap2(24), lap2(20, eps=0.05)):
        n = A.shape[0]
        S = strength(A)
        part = chunk_ids(n, K)
        cf1 = rs_partitioned(S, n, part)
        cf = pmis_stage(S, n, cf1, part)
        ST = transpose_lists(S, n)
        boundary = np.array([bool(np.any(part[S[i]] != part[i])) for i in range(n)])
        assert np.array_equal(cf[~boundary], cf1[~boundary])
        assert K > 1 or np.array_equal(cf, cf1)
        newc = (cf == C) & boundary
        for i in np.flatnonzero(newc):
            assert not np.any(newc[S[i]]), i
        for i in np.flatnonzero((cf == F) & boundary):
            assert np.any(cf[S[i]] == C) or len(ST[i]) == 0, i


@pytest.mark.parametrize("ranks", ["3", "2"])
def test_libpls_host_setup_bitwise_ranks(ranks):
    """hypre under mpirun -np G (pls.hypre_ranks): libpls's host setup equals
    the spec bit for bit with the per-rank HMIS first pass and inherited
    coarse ranks."""
    from lib.handle import boomeramg_host_level
    db = dict(INEXACT, **{"pls.hypre_ranks": ranks})
    for name, A in _blocks():
        A = A.tocsr()
        A.sort_indices()
        pc = PCBoomerAMG(A, db, "x_")
        for l, L in enumerate(pc.levels):
            nl, n, nc, cf, P = boomeramg_host_level(A, db, "x_", l)
            assert np.array_equal(cf, L["cf"].astype(np.int8)), (name, l)
            assert np.array_equal(P.data, L["P"].data), (name, l)
        assert not pc.levels or pc.levels[0]["parts"] is not None


def test_rank_partition_is_inherited():
    """Level 0 split as PETSc splits rows over 3 ranks; a coarse level's ranks own
    their C points; V-cycle PCG still converges."""
    A = lap2(24)
    three = PCBoomerAMG(A, dict(INEXACT, **{"pls.hypre_ranks": "3"}), "x_")
    assert three.levels[0]["parts"] == [192, 192, 192]
    for L, Ln in zip(three.levels, three.levels[1:]):
        assert sum(Ln["parts"]) == Ln["A"].shape[0] == int((L["cf"] == C).sum())
    b = np.random.default_rng(0).standard_normal(A.shape[0])
    assert pcg(A, b, three.apply) <= 14
