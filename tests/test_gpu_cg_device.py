"""The device-resident CG (runtime.cpp KSP::solve_cg_dev: the scalar
recurrences of KSPSolve_CG in a one-thread kernel, iterations enqueued in
batches with one read-back per batch) against the host-driven loop
(KSP::solve_cg, pls.cg_device 0): the same operations, so every inner solve's
iteration count and reason, the outer history and the solution are bitwise
equal -- including the ends a batch overruns (converged, max_it, indefinite
PC) where the extra enqueued iterations must leave x and r untouched."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))


@pytest.mark.parametrize("prob,pc", [("swelling", "diagonal"), ("footing", "undrained"),
                                     ("swelling", "diagonal 3-way")])
def test_cg_device_bitwise_harness(gpu, prob, pc):
    """The reference's inexact set at N = 10 (s / f / p CG + BoomerAMG with
    mpirun -np 8 semantics, CG + AMG in the fp fieldsplit's split 0)."""
    import robustness as R
    out = {}
    for dev in ("1", "0"):
        out[dev] = R.run_case(prob, 10, pc, "inexact", 8, extra={"pls.cg_device": dev}, history=True)
    a, b = out["1"], out["0"]
    assert a["its"] == b["its"] and a["reason"] == b["reason"]
    assert a["history"] == b["history"]
    assert a["inner"] == b["inner"]


@pytest.mark.parametrize("extra", [
    {"s_ksp_norm_type": "preconditioned"},
    {"s_ksp_max_it": "3"},             # every s solve ends at max_it inside a batch
    {"s_ksp_rtol": "1e-8"},            # long inner solves: batches of up to 32
])
def test_cg_device_bitwise_variants(gpu, extra):
    from lib.handle import Handle, params_to_options
    from oracle import synthetic as S
    spec = S.SynthSpec(2, 12)
    params = {"solver type": "gmres", "solver atol": 1e-10, "solver rtol": 1e-8, "solver maxiter": 200,
              "pc type": "diagonal", "inner ksp type": "preonly", "inner pc type": "ilu", "inner accel order": 0,
              "AAR order": 10, "AAR p": 5, "AAR omega": 1, "AAR beta": 1}
    db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right",
          "s_ksp_type": "cg", "s_pc_type": "jacobi", "s_ksp_rtol": "1e-3", "fp_ksp_type": "preonly",
          "fp_pc_type": "ilu", "pls.ksp_stats": "1"}
    db.update(extra)
    res = {}
    for dev in ("1", "0"):
        opts = dict(db, **{"pls.cg_device": dev})
        opts.update(params_to_options(params))
        h = Handle.synthetic(spec.dim, spec.N, spec.seed, spec.delta, opts)
        x, r = h.solve(S.rhs(spec))
        res[dev] = (x, r.its, r.reason, h.history(), h.ksp_stats("s_"))
        h.destroy()
    a, b = res["1"], res["0"]
    assert a[1] == b[1] and a[2] == b[2]
    assert np.array_equal(a[3], b[3])
    assert np.array_equal(a[0], b[0])
    assert tuple(a[4]) == tuple(b[4])
