"""Full-size GPU checks (BASELINE.json configs) through size-independent
properties -- the CPU oracle cannot run these sizes in test time.

* right-preconditioned GMRES's residual estimate |g_k| equals the true
  residual ||b - A x|| (unpreconditioned norm; computed on the device) to
  within accumulated rounding;
* bitwise reproducibility: two solves of the same system give the same
  history and solution (fixed-order reductions, no atomics in the Krylov path);
* the D16 SpMV layout agrees with the int32 SELL-64 layout to 1e-13 (lane-
  per-row slices bitwise, wide slices to summation-order rounding);
* the solve converges (reason 2); its iteration count and history are checked
  against the oracle at these sizes in ``tests/test_gpu_fullsize_oracle.py``.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _opts(nb_s, nb_fp, extra=None):
    o = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "s_ksp_type": "preonly", "s_pc_type": "bjacobi",
         "s_pc_bjacobi_blocks": str(nb_s), "fp_ksp_type": "preonly", "fp_pc_type": "bjacobi",
         "fp_pc_bjacobi_blocks": str(nb_fp), "pls.pc_type": "diagonal", "pls.solver_type": "gmres",
         "pls.solver_rtol": "1e-6", "pls.solver_atol": "1e-8", "pls.solver_maxiter": "100",
         "pls.inner_ksp_type": "preonly", "pls.inner_pc_type": "bjacobi"}
    o.update(extra or {})
    return o


@pytest.mark.parametrize("N,nb_s,nb_fp", [(27, 64, 64), (59, 256, 264)])
def test_full_size_properties(gpu, N, nb_s, nb_fp):
    import lib._native as Nt
    from lib.handle import Handle
    h = Handle.synthetic(3, N, 20261015, 0.05, _opts(nb_s, nb_fp))
    n = h.n
    b, x, r = Nt.DeviceArray(n), Nt.DeviceArray(n), Nt.DeviceArray(n)
    h.rhs_device(7, b.p)
    res = h.solve_device(b.p, x.p)
    hist = h.history()
    assert res.reason == 2
    h.matmult_device(x.p, r.p)
    bh, rh, xh = b.download(), r.download(), x.download()
    true = np.linalg.norm(bh - rh)
    assert abs(true - hist[-1]) <= 1e-3 * hist[-1], (true, hist[-1])
    assert hist[-1] <= 1e-6 * hist[0]
    # bitwise reproducibility
    x2 = Nt.DeviceArray(n)
    res2 = h.solve_device(b.p, x2.p)
    assert res2.its == res.its and np.array_equal(h.history(), hist) and np.array_equal(x2.download(), xh)
    # D16 vs int32 SELL-64 products
    h32 = Handle.synthetic(3, N, 20261015, 0.05, _opts(nb_s, nb_fp, {"pls.sell_d16": "0"}))
    assert h.spmv_layout()[0] and not h32.spmv_layout()[0]
    y32 = Nt.DeviceArray(n)
    h32.matmult_device(x.p, y32.p)
    assert np.max(np.abs(y32.download() - rh)) <= 1e-13 * np.max(np.abs(rh))
    for a in (b, x, r, x2, y32):
        a.free()
    h.destroy()
    h32.destroy()


def test_band_lu_footing_size():
    """Exact LU of the solid block of the footing configuration's 2-D N=128
    system (132,098 rows, 2,064 tile rows) through the band path: the 2-way
    PC with K_s exact and K_fp ILU(0) satisfies ||M y - x|| at rounding level
    for the block-lower M it applies (checked with the exported P on the host),
    and two applications agree bitwise (the flag-free granule sweeps sum in a
    fixed order whatever the timing)."""
    import lib._native as Nt  # noqa: F401
    from lib.handle import Handle
    import scipy.sparse as sp
    from oracle import native
    opts = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "s_ksp_type": "preonly", "s_pc_type": "lu",
            "fp_ksp_type": "preonly", "fp_pc_type": "ilu", "pls.lu_path": "band", "pls.pc_type": "diagonal",
            "pls.solver_type": "gmres", "pls.inner_ksp_type": "preonly", "pls.inner_pc_type": "lu"}
    h = Handle.synthetic(2, 128, 20261015, 0.05, opts)
    h.setup()
    n = h.n
    P = h.export_matrix(1).tocsr()
    ns = 2 * (2 * 128 + 1) ** 2
    Ks = P[:ns, :ns]
    x = np.random.default_rng(11).standard_normal(n)
    y = h.pc_apply(x)
    y2 = h.pc_apply(x)
    assert np.array_equal(y, y2)
    assert np.linalg.norm(Ks @ y[:ns] - x[:ns]) <= 1e-11 * np.linalg.norm(x[:ns])
    # the fp part is ILU(0) of K_fp applied to x_fp - P_fp,s y_s: check with the oracle's ILU(0)
    t = x[ns:] - P[ns:, :ns] @ y[:ns]
    f = native.ILU0(P[ns:, ns:].tocsr())
    assert np.linalg.norm(y[ns:] - f.solve(t)) <= 1e-12 * np.linalg.norm(y[ns:])
    h.destroy()


def test_full_size_three_way():
    """3-way block PC (FS + DIFF sweeps on two streams) at N=27 (~1M DoF):
    converges, GMRES estimate = device true residual, bitwise reproducible
    (the concurrent sweeps join before the w1/w2 combination, so stream timing
    cannot reorder any sum)."""
    import lib._native as Nt
    from lib.handle import Handle
    o = _opts(64, 64, {"pls.pc_type": "diagonal_3-way", "f_ksp_type": "preonly", "f_pc_type": "bjacobi",
                       "f_pc_bjacobi_blocks": "64", "p_ksp_type": "preonly", "p_pc_type": "bjacobi",
                       "p_pc_bjacobi_blocks": "8", "diff_ksp_type": "preonly", "diff_pc_type": "bjacobi",
                       "diff_pc_bjacobi_blocks": "8"})
    h = Handle.synthetic(3, 27, 20261015, 0.05, o)
    n = h.n
    b, x, r, x2 = (Nt.DeviceArray(n) for _ in range(4))
    h.rhs_device(7, b.p)
    res = h.solve_device(b.p, x.p)
    hist = h.history()
    assert res.reason == 2 and hist[-1] <= 1e-6 * hist[0]
    h.matmult_device(x.p, r.p)
    true = np.linalg.norm(b.download() - r.download())
    assert abs(true - hist[-1]) <= 1e-3 * hist[-1], (true, hist[-1])
    res2 = h.solve_device(b.p, x2.p)
    assert res2.its == res.its and np.array_equal(h.history(), hist) and np.array_equal(x2.download(), x.download())
    for a in (b, x, r, x2):
        a.free()
    h.destroy()


def test_gmres_longer_than_the_default_reduction_room():
    """A GMRES cycle longer than the context's default CGS reduction room
    (one partial per column and reduction block: 1024 x 136 doubles, i.e.
    ~560 columns at the 247 blocks of this 1.0M-row system): restart =
    maxit = 600 (footing.py's maxiter is 500, on 1.3M rows) runs to its last
    iteration with finite, non-increasing residual estimates (round 3: the
    buffer now grows with the restart length; before, the CGS partials of
    columns past ~450 of footing N=128 overran it and faulted the GPU)."""
    import lib._native as Nt
    from lib.handle import Handle
    opts = _opts(1, 1, {"s_pc_type": "jacobi", "fp_pc_type": "jacobi", "pls.inner_pc_type": "jacobi",
                        "pls.solver_rtol": "1e-300", "pls.solver_atol": "0", "pls.solver_maxiter": "600"})
    # pls.debug_bounds: a canary region behind the partials, checked after every KSP solve
    opts["pls.debug_bounds"] = "1"
    h = Handle.synthetic(3, 27, 20261015, 0.05, opts)
    n = h.n
    assert n >= 1_000_000
    b, x = Nt.DeviceArray(n), Nt.DeviceArray(n)
    h.rhs_device(7, b.p)
    res = h.solve_device(b.p, x.p)
    hist = h.history()
    assert res.its == 600 and res.reason < 0
    assert len(hist) == 601 and np.all(np.isfinite(hist)) and np.all(np.diff(hist) <= 0)
    assert np.all(np.isfinite(x.download()))
    b.free()
    x.free()
    h.destroy()


def _long_cycle(extra):
    import lib._native as Nt
    from lib.handle import Handle
    opts = _opts(1, 1, {"s_pc_type": "jacobi", "fp_pc_type": "jacobi", "pls.inner_pc_type": "jacobi",
                        "pls.solver_rtol": "1e-300", "pls.solver_atol": "0", "pls.solver_maxiter": "600"})
    opts.update(extra)
    h = Handle.synthetic(3, 8, 20261015, 0.05, opts)  # 30,207 rows: 8 reduction blocks
    b, x = Nt.DeviceArray(h.n), Nt.DeviceArray(h.n)
    try:
        h.rhs_device(7, b.p)
        return h.solve_device(b.p, x.p)
    finally:
        b.free()
        x.free()
        h.destroy()


def test_partials_overrun_is_caught():
    """The round-3 failure mode, reproduced inside the canary: the context's
    partials are capped at 100 doubles and not grown (the old fixed buffer,
    scaled down) so a 600-column CGS cycle needs 8 x 600.  Unguarded, the
    CGS partials of columns past 12 land in the canary region behind the
    buffer and check_bounds reports it; with the launch-site guard (the
    default) the first oversized launch throws before writing anything; with
    growth (the default) the same cycle runs to its end, canary intact."""
    base = {"pls.debug_bounds": "1", "pls.debug_partial_cap": "100", "pls.debug_no_grow": "1"}
    with pytest.raises(RuntimeError, match="canary"):
        _long_cycle(dict(base, **{"pls.debug_unguarded": "1"}))
    with pytest.raises(RuntimeError, match="reduction partials"):
        _long_cycle(base)
    res = _long_cycle({"pls.debug_bounds": "1", "pls.debug_partial_cap": "100"})
    assert res.its == 600
