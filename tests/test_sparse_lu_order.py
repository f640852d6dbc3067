"""Host-only checks of the sparse LU's ordering and symbolic analysis
(``pls_sparse_lu_analyze``; the MUMPS stand-in behind -pc_type lu,
petsc-options-exact:11-35, petsc-options-inexact:105-106; no device).

* the dissection is a permutation whose fronts are contiguous in postorder,
  children before parents;
* it is deterministic and independent of the host thread count;
* fill: the multilevel nested dissection (round 4, ``pls.lu_nd 1``, the
  default) reads fewer factor doubles per solve than round 3's level-set
  dissection and than SuperLU's minimum degree on A + A^T (scipy ``splu``,
  the independent check) on the footing system's blocks: the undrained
  solid block K_s and the fieldsplit's selfp Schur block of configs[2]'s
  option set;
* a front's update rows lie in ancestor fronts (the assembly tree property
  the multifrontal solve relies on).
"""
import numpy as np
import pytest
import scipy.sparse as sp


def _footing_blocks(N):
    from lib.fe_footing import assemble_footing
    from oracle.fieldsplit import selfp
    s = assemble_footing(N, "undrained")
    P = s.P.tocsr()
    iss = np.asarray(s.is_s)
    Ks = P[iss][:, iss].tocsr()
    fp = np.sort(np.concatenate([s.is_f, s.is_p]))
    Pfp = P[fp][:, fp].tocsr()
    ip, jf = np.searchsorted(fp, np.sort(s.is_p)), np.searchsorted(fp, np.sort(s.is_f))
    sub = lambda r, c: Pfp[r][:, c].tocsr()
    S = selfp(sub(ip, ip), sub(ip, jf), sub(jf, ip), sub(jf, jf))
    out = {}
    for name, M in (("Ks", Ks), ("schur", S), ("Kfp", Pfp)):
        M = M.tocsr()
        M.sort_indices()
        out[name] = M
    return out


@pytest.fixture(scope="module")
def blocks16():
    return _footing_blocks(16)


@pytest.mark.parametrize("name", ["Ks", "schur", "Kfp"])
@pytest.mark.parametrize("method", ["0", "1"])
def test_dissection_is_an_assembly_tree(blocks16, name, method):
    from lib.handle import sparse_lu_analyze
    M = blocks16[name]
    n = M.shape[0]
    st, perm, front_of, parent = sparse_lu_analyze(M, {"pls.lu_nd": method}, tree=True)
    assert np.array_equal(np.sort(perm), np.arange(n))
    assert np.all(np.diff(front_of) >= 0)  # fronts contiguous, numbered in postorder
    nf = int(st["fronts"])
    assert front_of[-1] == nf - 1 and parent[nf - 1] == -1
    assert np.all(parent[:-1] > np.arange(nf - 1))  # children before parents
    # the assembly tree property: every nonzero couples a front with an ancestor (or itself)
    pos = np.empty(n, dtype=np.int64)
    pos[perm] = np.arange(n)
    C = M.tocoo()
    nz = C.data != 0.0  # stored zeros are not structure (they add no fill)
    fa, fb = front_of[pos[C.row[nz]]], front_of[pos[C.col[nz]]]
    lo, hi = np.minimum(fa, fb), np.maximum(fa, fb)
    anc = lo.copy()
    for _ in range(int(st["levels"]) + 1):
        done = anc == hi
        anc = np.where(done | (anc < 0), anc, parent[np.maximum(anc, 0)])
    assert np.all(anc == hi)


def test_dissection_deterministic_across_thread_counts(blocks16):
    from lib.handle import sparse_lu_analyze
    M = blocks16["schur"]
    runs = [sparse_lu_analyze(M, {"pls.lu_nd_threads": t}, tree=True) for t in (1, 4, 4)]
    for st, perm, fo, par in runs[1:]:
        assert np.array_equal(perm, runs[0][1]) and np.array_equal(fo, runs[0][2]) and np.array_equal(par, runs[0][3])


@pytest.mark.parametrize("name", ["Ks", "schur"])
def test_multilevel_fill_beats_level_sets_and_minimum_degree(blocks16, name):
    import scipy.sparse.linalg as spl
    from lib.handle import sparse_lu_analyze
    M = blocks16[name]
    ml = sparse_lu_analyze(M, {"pls.lu_nd": "1"})
    ls = sparse_lu_analyze(M, {"pls.lu_nd": "0"})
    lu = spl.splu(M.tocsc(), permc_spec="MMD_AT_PLUS_A", options=dict(SymmetricMode=True))
    mmd = lu.L.nnz + lu.U.nnz
    # dense fronts count their explicit zeros too, so this favours minimum degree
    assert ml["solve_doubles"] <= 0.75 * ls["solve_doubles"], (ml, ls)
    assert ml["solve_doubles"] <= 1.25 * mmd, (ml["solve_doubles"], mmd)
    assert ml["flops"] < ls["flops"]
