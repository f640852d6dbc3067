"""BASELINE.json configurations beyond the headline, on the GPU.

* configs[2] ``footing-inexact-ilu`` (footing.py N=128, petsc-options-inexact
  with BJACOBI(ILU(0)) blocks in place of BoomerAMG): the option set bench.py
  runs (``bench.solver_options`` with the preset) compared with the oracle at
  the configuration's own size, 2-D N=128 (280,837 DoF), and at N=16.  The
  outer GMRES contains inner CG solves (rtol 1e-1 / 1e-4) and a Schur
  fieldsplit with an inner CG on split 0: a nonlinear preconditioner inside
  non-flexible GMRES, so rounding differences are amplified; the bound is
  max(1e-10, 10x the oracle's own history deviation under 1e-15 relative
  perturbations of its inner PC outputs) -- measured, not assumed
  (``_self_sensitivity``).  Iteration count and reason exact.
* configs[4] ``aar-m5`` (AAR depth m=5, p=5; reference ``lib/AAR.py:46-128``
  driven by ``swelling-3d.py``'s parameters): 3-D N=4 and N=8 against the
  oracle; at the metric size (3-D N=59, bench's block counts) through
  properties -- convergence, bitwise reproducibility across fresh handles, and
  the returned x reproduces the history's definition ||M^-1 (b - A x)||.
"""
import os
import sys

import numpy as np
import pytest

from oracle import synthetic as S
from test_gpu_parity import _compare_solve

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _bench_options(argv):
    """(params, db) exactly as bench.py builds them for these flags."""
    import argparse
    import bench
    ap = argparse.Namespace()
    cfg = dict(bench.CONFIGS[argv["config"]])
    defaults = dict(dim=3, atol=1e-8, aar_order=10, inner="bjacobi", inexact=False, blocks_s=256, blocks_fp=264,
                    blocks_p=11, blocks_inner=64, maxit=100, pc_type="diagonal", solver="gmres")
    defaults.update({k: v for k, v in cfg.items() if k not in ("preset", "cpu_N", "N")})
    defaults.update(argv.get("override", {}))
    for k, v in defaults.items():
        setattr(ap, k, v)
    ap.preset = cfg.get("preset")
    return bench.solver_options(ap)


@pytest.mark.parametrize("N", [16, 128])
def test_footing_inexact_ilu_vs_oracle(gpu, N):
    params, db = _bench_options({"config": "footing-inexact-ilu"})
    assert params["solver atol"] == 1e-4 and params["solver maxiter"] == 500
    assert db["fp_pc_fieldsplit_type"] == "schur" and db["s_pc_type"] == "bjacobi"
    r, o = _compare_solve(S.SynthSpec(2, N), params, db=db, sensitivity=True)
    assert r.reason in (2, 3)


@pytest.mark.parametrize("N", [4, 8])
def test_aar_m5_3d_vs_oracle(gpu, N):
    params, db = _bench_options({"config": "aar-m5", "override": {"blocks_s": 4, "blocks_fp": 4}})
    assert params["solver type"] == "aar" and params["AAR order"] == 5 and params["AAR p"] == 5
    r, o = _compare_solve(S.SynthSpec(3, N), dict(params, **{"solver maxiter": 200}), db=db)
    assert r.reason == 2


def test_aar_m5_full_size_properties(gpu):
    """History entry k of AAR is ||M^-1 (b - A x_{k-1})|| (the iterate before
    the k-th update, AAR.py:75-78,117), so the returned x is checked through a
    second, fresh handle run one iteration further: its first its + 1 entries
    are bitwise those of the first run (fixed-order arithmetic), and its last
    entry equals ||M^-1 (b - A x)|| recomputed on the device from the first
    run's x."""
    import lib._native as Nt
    from lib.handle import Handle, params_to_options
    params, db = _bench_options({"config": "aar-m5"})
    opts = dict(db)
    opts.update(params_to_options(params))
    h = Handle.synthetic(3, 59, 20261015, 0.05, opts)
    n = h.n
    b, x, x2, r, z = (Nt.DeviceArray(n) for _ in range(5))
    h.rhs_device(7, b.p)
    res = h.solve_device(b.p, x.p)
    hist = np.asarray(h.history())
    assert res.reason == 2 and hist[-1] <= 1e-6 * hist[0]
    h.matmult_device(x.p, r.p)
    z.upload(b.download() - r.download())
    h.pc_apply_device(z.p, r.p)
    true = np.linalg.norm(r.download())
    h.destroy()
    # (AAR's F / X histories persist across solves of one handle, AAR.py:20-22:
    # the second run needs a fresh handle)
    opts2 = dict(opts, **{"pls.solver_maxiter": str(res.its + 1), "pls.solver_rtol": "1e-300",
                          "pls.solver_atol": "0"})
    h2 = Handle.synthetic(3, 59, 20261015, 0.05, opts2)
    res2 = h2.solve_device(b.p, x2.p)
    hist2 = np.asarray(h2.history())
    assert res2.its == res.its + 1
    assert np.array_equal(hist2[:res.its + 1], hist)
    assert abs(hist2[-1] - true) <= 1e-10 * true, (hist2[-1], true)
    for a in (b, x, x2, r, z):
        a.free()
    h2.destroy()
