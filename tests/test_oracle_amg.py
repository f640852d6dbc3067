"""CPU tests of the AMG specification (oracle/amg.py), the stand-in for
BoomerAMG (-pc_type hypre) and the restatement behind -pc_type gamg.

hypre is absent from this image and from the reference tree, so nothing here
can be pinned against the reference's own numbers ("parity unpinned", see
DESIGN.md): these are known-answer tests of the aggregation on hand-checked
graphs and property tests of the multigrid cycle (symmetry, convergence
factor, option mapping).  The device implementation is compared with this
oracle in tests/test_gpu_amg.py.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle.amg import PCAMG, aggregate, power_lambda
from oracle.petsc import make_pc_of_type


def lap1(n):
    return sp.diags([-1.0, 2.0, -1.0], [-1, 0, 1], shape=(n, n)).tocsr()


def lap2(n):
    I, T = sp.eye(n), lap1(n)
    return (sp.kron(I, T) + sp.kron(T, I)).tocsr()


def pcg(A, b, M, rtol=1e-8, maxit=500):
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
            return k + 1, x
        z = M(r)
        rzn = r @ z
        p = z + rzn / rz * p
        rz = rzn
    return maxit, x


def test_aggregate_chain_kat():
    # pass 1: 0 takes {0,1}; 2 is blocked (1 taken); 3 takes {2,3,4}; 5 blocked
    # pass 2: 5 joins 4's aggregate
    agg, na = aggregate(lap1(6))
    assert na == 2
    assert agg.tolist() == [0, 0, 1, 1, 1, 1]


def test_aggregate_pass2_tie_takes_smallest_neighbour():
    # path 0-1-2-3-4 plus a node 5 coupled equally to 1 and 4
    A = lap1(5).tolil()
    A.resize((6, 6))
    A[5, 5] = 2.0
    for j in (1, 4):
        A[5, j] = A[j, 5] = -1.0
    agg, na = aggregate(A.tocsr())
    # pass 1: row 0 -> {0,1}; row 2 blocked by 1; row 3 -> {2,3,4}; row 5 blocked (1, 4 taken)
    # pass 2: row 5 ties between 1 (agg 0) and 4 (agg 1) -> smallest j = 1
    assert agg.tolist() == [0, 0, 1, 1, 1, 0]
    assert na == 2


def test_aggregate_singletons_and_threshold():
    # diagonal matrix: no strong neighbours -> every row its own aggregate
    agg, na = aggregate(sp.eye(5).tocsr())
    assert na == 5 and agg.tolist() == [0, 1, 2, 3, 4]
    # anisotropic 2-D operator: with theta 0.25 the weak (eps) direction is
    # dropped, aggregates become lines along the strong direction
    n, eps = 6, 1e-3
    I = sp.eye(n)
    A = (sp.kron(I, lap1(n)) + eps * sp.kron(lap1(n), I)).tocsr()
    agg0, na0 = aggregate(A, 0.0)
    agg1, na1 = aggregate(A, 0.25)
    assert na1 > na0
    grid = agg1.reshape(n, n)  # row = weak index, column = strong index
    for r in range(n):  # no aggregate spans two weak-direction lines
        for s in range(r + 1, n):
            assert not set(grid[r]) & set(grid[s])


def test_aggregates_cover_and_are_connected():
    A = lap2(9)
    agg, na = aggregate(A)
    assert agg.min() == 0 and agg.max() == na - 1
    G = (abs(A) + abs(A).T).tolil()
    G.setdiag(0)
    G = G.tocsr()
    for a in range(na):
        nodes = np.flatnonzero(agg == a)
        seen, todo = {nodes[0]}, [nodes[0]]
        members = set(nodes.tolist())
        while todo:
            i = todo.pop()
            for j in G.indices[G.indptr[i]:G.indptr[i + 1]]:
                if j in members and j not in seen:
                    seen.add(j)
                    todo.append(j)
        assert seen == members, f"aggregate {a} is not connected"


def test_power_lambda_bounds():
    A = lap2(16)
    lam = power_lambda(A, 1.0 / A.diagonal())
    assert 1.5 < lam <= 2.0 + 1e-12  # spectrum of D^-1 A for the 5-point Laplacian is in (0, 2)


def test_hierarchy_shape_and_coarse_limit():
    pc = PCAMG(lap2(40))
    sizes = [L["A"].shape[0] for L in pc.levels] + [pc.coarse.shape[0]]
    assert sizes[0] == 1600
    assert all(a > b for a, b in zip(sizes, sizes[1:]))
    assert sizes[-1] <= 50
    for L in pc.levels:  # Galerkin: R = P^T exactly
        assert (L["R"] != L["P"].T).nnz == 0
    # -pc_mg_levels caps the depth, -pc_gamg_coarse_eq_limit the coarse size
    assert len(PCAMG(lap2(40), {"pc_mg_levels": "2"}).levels) == 1
    assert PCAMG(lap2(40), {"pc_gamg_coarse_eq_limit": "2000"}).levels == []


def test_vcycle_is_symmetric_and_spd():
    A = lap2(24)
    pc = PCAMG(A)
    rng = np.random.default_rng(1)
    u, v = rng.standard_normal((2, A.shape[0]))
    Mu, Mv = pc.apply(u), pc.apply(v)
    assert abs(u @ Mv - v @ Mu) <= 1e-12 * abs(u @ Mv)
    assert u @ Mu > 0 and v @ Mv > 0


def test_amg_cg_beats_jacobi_and_scales():
    its = []
    for n in (32, 64):
        A = lap2(n)
        b = np.random.default_rng(0).standard_normal(A.shape[0])
        k_amg, x = pcg(A, b, PCAMG(A).apply)
        assert np.linalg.norm(b - A @ x) <= 1e-8 * np.linalg.norm(b)
        k_jac, _ = pcg(A, b, lambda r: r / 4.0)
        assert k_amg * 5 < k_jac
        its.append(k_amg)
    assert its[1] <= its[0] + 4  # near mesh-independent


def test_hypre_standin_sweeps_option():
    A = lap2(20)
    assert PCAMG(A, {}, "s_", hypre=True).K == 1
    assert PCAMG(A, {"s_pc_hypre_boomeramg_grid_sweeps_all": "3"}, "s_", hypre=True).K == 3
    assert PCAMG(A, {"s_mg_levels_ksp_max_it": "4"}, "s_", hypre=True).K == 4
    assert PCAMG(A, {}, "s_").K == 2
    assert make_pc_of_type("hypre", A, {}, "s_").K == 1
    with pytest.raises(NotImplementedError):
        make_pc_of_type("hypre", A, {"pls.hypre": "error"}, "s_")


def test_small_and_empty():
    A = lap1(10)  # below the coarse limit: one level, exact solve
    pc = PCAMG(A)
    assert pc.levels == []
    b = np.arange(10.0)
    assert np.allclose(A @ pc.apply(b), b)
    assert PCAMG(sp.csr_matrix((0, 0))).apply(np.zeros(0)).size == 0
