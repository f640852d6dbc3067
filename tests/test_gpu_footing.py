"""configs[2] on its true matrices: the footing system (lib/fe_footing.py --
footing.py's twice locally refined mesh, top traction, footing BCs,
"pc type" undrained) solved by libpls.so on the GPU against the oracle on the
same CSR.

* the option sets: petsc-options-exact (PREONLY + LU), configs[2]'s
  petsc-options-inexact with BJACOBI(ILU(0)) for BoomerAMG (bench's
  ``footing-inexact-ilu`` preset; inner CG, Schur lower/selfp fieldsplit on
  fp), and petsc-options-inexact itself (hypre -> the classical AMG);
* bounds as tests/test_gpu_fe.py's ``_compare``: iteration count and reason
  exact, history within max(1e-10, 10x the oracle's own rounding noise
  floor), solution likewise, true residual for linear PCs.  The noise floor
  here also includes the oracle's deviation when its LU is swapped for the
  same LU under another column ordering (``_lu_swap_floor``): footing's
  undrained solid block (ks div div over E = 3e4) is ill-conditioned enough
  that two exact solvers differ by ~cond eps -- measured 1.5e-7 .. 2.8e-7 in
  the history at N = 8, undrained, LU; the device sat at 2.5e-7.
  footing.py's own "pc type" is undrained; "diagonal" does not converge on
  this system (500 its) and "undrained 3-way"'s iteration count moves under
  that swap (148 vs 150-153), so neither is a parity case;
* the committed footing fixtures (tests/golden/footing/) reproduced by the
  device -- its, reason, history and x;
* larger solves, N = 32, through properties (converged, bitwise
  reproducible, true residual of the returned x): the exact option set, and
  footing.py's own (petsc-options-inexact, hypre -> the classical AMG with
  hybrid Gauss-Seidel over 256-chunk partitions).
"""
import json
import os

import numpy as np
import pytest

from lib import fe_footing as FF
from test_gpu_fe import _compare

pytestmark = pytest.mark.gpu

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _options(preset, pc="undrained"):
    import sys
    sys.path.insert(0, HERE)
    import make_golden_footing as G
    return G.options(preset, pc)


@pytest.mark.parametrize("N,pc,preset", [
    (8, "undrained", "exact"),
    (16, "undrained", "exact"),
    (8, "diagonal 3-way", "exact"),
    (8, "undrained", "inexact-ilu"),
    (8, "undrained", "inexact"),
    (12, "undrained", "inexact"),
    (16, "undrained", "inexact"),
])
def test_footing_vs_oracle(gpu, N, pc, preset):
    s = FF.assemble_footing(N, pc)
    params, db = _options(preset, pc)
    r = _compare(s, params, db, linear_pc=preset == "exact", lu_swap=True)
    assert r.reason > 0


def test_inner_cg_indefinite_pc_abort(gpu):
    """N = 12, configs[2]'s inexact-ILU set: ILU(0) blocks of the undrained
    solid block are indefinite, and PETSc's CG (cg.c) stops the inner solve
    with KSP_DIVERGED_INDEFINITE_PC after ~4 iterations instead of iterating
    to max_it.  The device block PC (inner CG + BJACOBI(ILU(0)), Schur
    fieldsplit on fp) against the oracle's on the same vectors."""
    from lib.handle import Handle, params_to_options
    from oracle.solver import OracleSolver
    s = FF.assemble_footing(12, "undrained")
    params, db = _options("inexact-ilu")
    o = OracleSolver(s.A, s.P, s.P_diff, s.is_s, s.is_f, s.is_p, params, db, s.bcs_sub_pressure)
    opts = dict(db)
    opts.update(params_to_options(params))
    h = Handle.from_csr(s.A, s.P, s.P_diff, s.is_s, s.is_f, s.is_p, s.bcs_sub_pressure, opts)
    rng = np.random.default_rng(4)
    aborted = 0
    for x in (s.b, rng.standard_normal(s.A.shape[0])):
        yo = o.block_pc.apply(x)
        aborted += o.block_pc.ksp_s.reason == -8
        y = h.pc_apply(x)
        assert np.max(np.abs(y - yo)) <= 1e-8 * np.max(np.abs(yo))
    assert aborted >= 1
    h.destroy()


@pytest.mark.parametrize("name", ["footing_N8_undrained_exact", "footing_N8_undrained_inexact_ilu",
                                  "footing_N8_3way_exact"])
def test_device_reproduces_footing_golden(gpu, name):
    z = np.load(os.path.join(HERE, "footing", name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    s = FF.assemble_footing(meta["N"], meta["pc"])
    r, hist, x, tol = _compare(s, meta["params"], meta["db"], linear_pc=meta["preset"] == "exact", full=True,
                               lu_swap=True)
    assert r.its == int(z["its"]) and r.reason == int(z["reason"])
    hz, xz = np.asarray(z["history"]), np.asarray(z["x"])
    assert np.max(np.abs(hist - hz) / np.abs(hz)) <= tol
    assert np.linalg.norm(x - xz) <= max(1e-8, tol) * np.linalg.norm(xz)


def test_footing_full_solve_properties(gpu):
    """The assembled N = 32 system (79,104 DoF) with the exact option set
    (PREONLY + LU; the s block and the fp block by the band LU): converges,
    two fresh handles give bitwise equal histories and solutions, and the
    true residual ||b - A x|| of the returned x matches the last GMRES
    estimate (a linear PC).  footing.py's own AMG set is parity-tested at
    N = 8 above; at N = 32 its device solve exceeded the test budget (the
    classical AMG's latency-bound level sweeps), and configs[2]'s
    N = 128 is bench-only (setup ~18 s since round 4; a solve to 500 its
    takes ~270 s)."""
    from lib.handle import Handle, params_to_options
    s = FF.assemble_footing(32, "undrained")
    assert s.A.shape[0] == 79_104
    params, db = _options("exact")
    opts = dict(db)
    opts.update(params_to_options(params))
    runs = []
    for _ in range(2):
        h = Handle.from_csr(s.A, s.P, s.P_diff, s.is_s, s.is_f, s.is_p, s.bcs_sub_pressure, opts)
        x, r = h.solve(s.b)
        runs.append((r, h.history(), x))
        h.destroy()
    (r1, h1, x1), (r2, h2, x2) = runs
    assert r1.reason > 0 and r1.its == r2.its
    assert np.array_equal(h1, h2) and np.array_equal(x1, x2)
    assert h1[-1] <= max(params["solver rtol"] * h1[0], params["solver atol"])
    true_r = np.linalg.norm(s.b - s.A @ x1)
    assert abs(true_r - h1[-1]) <= 1e-2 * h1[-1] + 1e-12 * np.linalg.norm(s.b)


def test_footing_amg_solve_properties(gpu):
    """footing.py's own option set (petsc-options-inexact, BoomerAMG -> the
    classical AMG, hybrid Gauss-Seidel in chunks, sparse LU on the Schur split)
    on the N = 32 system (79,104 DoF), 60 outer iterations: two fresh handles
    give bitwise equal histories and solutions (the nonlinear inner CG is
    deterministic), the GMRES estimate decreases from the first iteration, and
    the whole run stays inside the test budget.  From N = 24 on, the inner CG
    on the undrained solid block occasionally stalls (oracle, N = 24: 67 outer
    its, inner solves of up to 815 its and one KSP_DIVERGED_INDEFINITE_PC; the
    device at N = 32: one inner solve at PETSc's max_it 10,000 within 40 outer
    its) -- the configuration's own behaviour, parity-tested at N = 8..16."""
    import time
    from lib.handle import Handle, params_to_options
    s = FF.assemble_footing(32, "undrained")
    params, db = _options("inexact")
    params = dict(params, **{"solver maxiter": 60})
    opts = dict(db)
    opts.update(params_to_options(params))
    runs = []
    t0 = time.perf_counter()
    for _ in range(2):
        h = Handle.from_csr(s.A, s.P, s.P_diff, s.is_s, s.is_f, s.is_p, s.bcs_sub_pressure, opts)
        x, r = h.solve(s.b)
        runs.append((r, h.history(), x))
        h.destroy()
    dt = time.perf_counter() - t0
    print(f"footing N=32 AMG: {runs[0][0].its} its, reason {runs[0][0].reason}, {dt:.1f} s for two setups + solves")
    (r1, h1, x1), (r2, h2, x2) = runs
    assert r1.its == r2.its and r1.reason == r2.reason
    assert np.array_equal(h1, h2) and np.array_equal(x1, x2)
    assert np.all(np.isfinite(h1)) and h1[-1] < h1[0]
    assert dt < 240


def test_footing_N128_configs2_setup_and_iterations(gpu):
    """configs[2] at its named size on its true matrices (1,308,592 DoF) with
    footing.py's own option set: the whole setup (five classical-AMG
    hierarchies, the sparse LU of the 615,714-row Schur split) within 60 s,
    10 outer GMRES iterations whose estimates never increase, and the block
    PC bitwise repeatable (two applications of the same vector).  A full
    solve is dominated by inner CG solves of the undrained solid block that
    stall at max_it."""
    import time
    from lib.handle import Handle, params_to_options
    s = FF.assemble_footing(128, "undrained")
    assert s.A.shape[0] == 1_308_592
    params, db = _options("inexact")
    params = dict(params, **{"solver maxiter": 10})
    opts = dict(db)
    opts.update(params_to_options(params))
    t0 = time.perf_counter()
    h = Handle.from_csr(s.A, s.P, s.P_diff, s.is_s, s.is_f, s.is_p, s.bcs_sub_pressure, opts)
    h.setup()
    h.create_solver()
    t_setup = time.perf_counter() - t0
    print(f"footing N=128 setup {t_setup:.1f} s")
    assert t_setup < 60
    x, r = h.solve(s.b)
    hist = h.history()
    assert r.its == 10 and np.all(np.isfinite(hist)) and np.all(np.diff(hist) <= 0)
    v = np.random.default_rng(0).standard_normal(s.A.shape[0])
    assert np.array_equal(h.pc_apply(v), h.pc_apply(v))
    h.destroy()
