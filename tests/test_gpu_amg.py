"""GPU parity of the device AMG (csrc/amg.cpp) against its specification
oracle/amg.py: -pc_type gamg, and -pc_type hypre (the BoomerAMG stand-in the
reference's drivers and petsc-options-inexact select).

Tolerances:
  * one block-preconditioner application: <= 1e-12 relative (the hierarchy is
    built bit-identically on the host; only the device V-cycle's summation
    order differs, amplified by the cycle's norm);
  * solves: identical iteration count and reason; residual histories within
    1e-10 relative for linear inner solves (PREONLY + AMG), and within 10x the
    oracle's own rounding sensitivity for inner CG (a nonlinear PC inside
    outer GMRES; see test_gpu_parity._compare_solve).
BoomerAMG itself is absent from this image: iteration counts match this
specification, not hypre ("parity unpinned" against the reference).
"""
import numpy as np
import pytest

from oracle import synthetic as S
from test_gpu_parity import BASE, ILU_DB, _compare_solve, _handle, _oracle

pytestmark = pytest.mark.gpu

PREFIXES = ("s_", "f_", "p_", "diff_", "fp_")

# petsc-options-inexact (reference) option set: CG + BoomerAMG on s/f/p,
# PREONLY + BoomerAMG on diff, Schur fieldsplit (lower, selfp) on fp with
# CG + BoomerAMG on split 0 and LU on the Schur split
INEXACT = {
    "global_ksp_type": "gmres", "global_ksp_norm_type": "unpreconditioned",
    "s_ksp_type": "cg", "s_ksp_norm_type": "unpreconditioned", "s_ksp_atol": "0.0", "s_ksp_rtol": "1e-1",
    "s_pc_type": "hypre", "s_pc_hypre_boomeramg_grid_sweeps_all": "1",
    "f_ksp_type": "cg", "f_ksp_norm_type": "unpreconditioned", "f_ksp_atol": "0.0", "f_ksp_rtol": "1e-2",
    "f_pc_type": "hypre", "f_pc_hypre_boomeramg_grid_sweeps_all": "1",
    "p_ksp_type": "cg", "p_ksp_norm_type": "unpreconditioned", "p_ksp_atol": "0.0", "p_ksp_rtol": "1e-2",
    "p_pc_type": "hypre",
    "diff_ksp_type": "preonly", "diff_pc_type": "hypre",
    "fp_ksp_type": "preonly", "fp_ksp_rtol": "1e-2", "fp_ksp_atol": "0.0",
    "fp_pc_fieldsplit_type": "schur", "fp_pc_fieldsplit_schur_fact_type": "lower",
    "fp_pc_fieldsplit_schur_precondition": "selfp",
    "fp_fieldsplit_0_ksp_type": "cg", "fp_fieldsplit_0_ksp_rtol": "1e-4", "fp_fieldsplit_0_ksp_atol": "0.0",
    "fp_fieldsplit_0_ksp_max_it": "10", "fp_fieldsplit_0_pc_type": "hypre",
    "fp_fieldsplit_1_ksp_type": "preonly", "fp_fieldsplit_1_pc_type": "lu",
}
INEXACT_PARAMS = {"inner ksp type": "cg", "inner pc type": "hypre", "solver maxiter": 200}


def _amg_db(t, extra=None):
    """AMG on the s/f/p/diff blocks; the coupled (indefinite) 2-way fp block keeps ILU(0)."""
    db = dict(ILU_DB)
    for pre in PREFIXES:
        db[pre + "pc_type"] = t if pre != "fp_" else "ilu"
    db.update(extra or {})
    return db


@pytest.mark.parametrize("spec", [S.SynthSpec(2, 16), S.SynthSpec(3, 5)], ids=["2d16", "3d5"])
@pytest.mark.parametrize("pc_type", ["diagonal", "diagonal 3-way"])
@pytest.mark.parametrize("t", ["gamg", "hypre"])
def test_amg_pc_apply_matches_oracle(gpu, spec, pc_type, t):
    params = dict(BASE, **{"pc type": pc_type, "inner pc type": "lu"})
    db = _amg_db(t)
    h = _handle(spec, params, db)
    o = _oracle(spec, params, db)
    rng = np.random.default_rng(3)
    x = rng.standard_normal(spec.n)
    y = h.pc_apply(x)
    yo = o.block_pc.apply(x)
    assert np.max(np.abs(y - yo)) <= 1e-12 * np.max(np.abs(yo))


@pytest.mark.parametrize("pc_type", ["diagonal", "diagonal 3-way"])
def test_gmres_preonly_gamg(gpu, pc_type):
    """Linear inner solves: the strict 1e-10 history bound."""
    _compare_solve(S.SynthSpec(2, 16), {"pc type": pc_type, "inner pc type": "lu"}, db=_amg_db("gamg"))


def test_gmres_preonly_gamg_options(gpu):
    db = _amg_db("gamg", {"s_mg_levels_ksp_max_it": "3", "s_pc_gamg_threshold": "0.05",
                          "f_pc_gamg_coarse_eq_limit": "200", "p_pc_mg_levels": "2"})
    _compare_solve(S.SynthSpec(2, 16), {"pc type": "diagonal 3-way", "inner pc type": "lu"}, db=db)


@pytest.mark.parametrize("pc_type", ["diagonal", "diagonal 3-way"])
def test_reference_inexact_option_set(gpu, pc_type):
    """The reference's petsc-options-inexact configuration end to end (BoomerAMG -> AMG stand-in)."""
    _compare_solve(S.SynthSpec(2, 12), dict(INEXACT_PARAMS, **{"pc type": pc_type}), db=dict(INEXACT),
                   sensitivity=True)


def test_inexact_3d(gpu):
    _compare_solve(S.SynthSpec(3, 4), dict(INEXACT_PARAMS, **{"pc type": "diagonal 3-way"}), db=dict(INEXACT),
                   sensitivity=True)


def test_hypre_is_the_default_inner_pc(gpu):
    """No s_/f_/p_/diff_ pc options: the reference drivers' "inner pc type": "hypre" default."""
    db = {k: v for k, v in INEXACT.items() if not k.endswith("pc_type") or k.startswith("fp_")}
    _compare_solve(S.SynthSpec(2, 10), dict(INEXACT_PARAMS, **{"pc type": "diagonal 3-way"}), db=db,
                   sensitivity=True)


def test_hypre_error_option(gpu):
    spec = S.SynthSpec(2, 4)
    h = _handle(spec, BASE, dict(ILU_DB, s_pc_type="hypre", **{"pls.hypre": "error"}))
    with pytest.raises(RuntimeError, match="hypre"):
        h.setup()


def test_amg_larger_hierarchy(gpu):
    """Two coarse levels on the solid block (3-D, N = 12)."""
    spec = S.SynthSpec(3, 12)
    params = dict(BASE, **{"pc type": "diagonal 3-way", "inner pc type": "lu"})
    db = _amg_db("gamg")
    h = _handle(spec, params, db)
    o = _oracle(spec, params, db)
    assert len(o.block_pc.ksp_s.pc.levels) >= 2
    x = np.random.default_rng(5).standard_normal(spec.n)
    y, yo = h.pc_apply(x), o.block_pc.apply(x)
    assert np.max(np.abs(y - yo)) <= 1e-12 * np.max(np.abs(yo))
