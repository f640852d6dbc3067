"""Why the reference's inexact s-block CG stalls (VERDICT r05
item 1), pinned on the CPU oracle at footing N = 10.

The inexact set solves the solid block with CG + BoomerAMG
(petsc-options-inexact:12-24).  The block the reference hands it comes from
dolfin's ``bc.apply`` (lib/Poromechanics.py:76-78): Dirichlet rows replaced by
identity rows, their columns kept, so it is not symmetric.  With a right-hand
side that is nonzero on the constrained rows -- what the outer GMRES's Krylov
vectors carry after the first iterations -- CG on that block does not converge
(max_it, or an indefinite preconditioner: the V-cycle built on the
nonsymmetric block is not SPD either); with the constrained columns
eliminated too (symmetric) the same CG + the same AMG converges in ~6-11
iterations.  So the stall is the reference's own method, not the AMG stand-in
(tools/s_cg_attribution.py: the same at footing N = 20 and swelling N = 40,
profiles/r06_s_cg_attribution.jsonl)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "poroelasticity-linear-solvers_amd"), os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)


@pytest.fixture(scope="module")
def blocks():
    import s_cg_attribution as T
    from lib.fe_footing import assemble_footing
    from robustness import load_set
    s = assemble_footing(10, "undrained")
    K, _ = T.s_block(s)
    bc = T.identity_rows(K)
    return T, K, T.symmetrized(K, bc), bc, load_set("inexact")


@pytest.mark.parametrize("nranks", [8, 1])
def test_symmetric_block_converges(blocks, nranks):
    T, K, Ks, bc, db = blocks
    assert bc.size > 0
    dbn = dict(db, **({"pls.hypre_ranks": "8", "pls.hypre_relax_chunks": "8"} if nranks > 1
                      else {"pls.hypre_relax_chunks": "1"}))
    r = np.random.default_rng(1).standard_normal(K.shape[0])
    res = T.run(Ks, r, dbn, 200)
    assert res["reason"] > 0 and res["its"] <= 15, res


@pytest.mark.parametrize("nranks", [8, 1])
def test_bc_apply_block_stalls(blocks, nranks):
    T, K, Ks, bc, db = blocks
    assert abs(K - K.T).sum() > 0  # bc.apply's rows-only elimination: not symmetric
    dbn = dict(db, **({"pls.hypre_ranks": "8", "pls.hypre_relax_chunks": "8"} if nranks > 1
                      else {"pls.hypre_relax_chunks": "1"}))
    r = np.random.default_rng(1).standard_normal(K.shape[0])
    res = T.run(K, r, dbn, 200)
    assert res["reason"] < 0, res  # max_it (-3) or indefinite PC (-8), never converged
