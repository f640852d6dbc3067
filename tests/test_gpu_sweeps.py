"""ILU(0) sweep kernels on blocks sized to their limits.

The window sweep (k_ilu_blocks_window) keeps a block's per-window stream
offsets in registers; blocks of up to ilu_window_max_rows() = 19,904 rows
(311 windows) qualify.  Round 4 held only 192 offsets, so a block of more
than 12,224 rows read wrong offsets.  Here a one-block ILU(0) on a 19,880-row
s block (311 windows) and a 12,300-row fp block is forced onto the window
sweep and compared against the workgroup sweep and the oracle
(lib/Preconditioner.py:219-246's 2-way apply; ILU(0) natural order,
PETSc's PCILU).  The sweep chosen is read from pls.ilu_view's line, so the
test fails if the window path was not the one that ran.

Matrices: 5-point-stencil blocks on 2-D grids (natural order: one entry per
row outside the 64-row window in each triangle), random nonsymmetric values,
strictly diagonally dominant, weak field coupling.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle.solver import OracleSolver

pytestmark = pytest.mark.gpu

PARAMS = {"solver type": "gmres", "solver atol": 1e-8, "solver rtol": 1e-6, "solver maxiter": 100,
          "pc type": "diagonal", "inner ksp type": "preonly", "inner pc type": "ilu", "inner accel order": 0,
          "AAR order": 10, "AAR p": 5, "AAR omega": 1, "AAR beta": 1}
DB = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "s_ksp_type": "preonly", "s_pc_type": "ilu",
      "fp_ksp_type": "preonly", "fp_pc_type": "ilu", "pls.ilu_view": "1"}


def _grid_block(nx, ny, rng):
    n = nx * ny
    i = np.arange(n)
    rows, cols = [i], [i]
    for d, ok in ((1, (i % nx) < nx - 1), (-1, (i % nx) > 0), (nx, i < n - nx), (-nx, i >= nx)):
        rows.append(i[ok])
        cols.append(i[ok] + d)
    r, c = np.concatenate(rows), np.concatenate(cols)
    v = -rng.uniform(0.2, 1.0, r.size)
    v[:n] = 0.0
    M = sp.csr_matrix((v, (r, c)), shape=(n, n))
    M = M + sp.diags(np.asarray(abs(M).sum(axis=1)).ravel() + rng.uniform(0.05, 0.5, n))
    return M.tocsr()


def _system():
    rng = np.random.default_rng(31)
    Ks = _grid_block(140, 142, rng)  # 19,880 rows: 311 windows
    Kf = _grid_block(90, 100, rng)   # 9,000
    Kp = _grid_block(60, 55, rng)    # 3,300
    ns, nf, npr = Ks.shape[0], Kf.shape[0], Kp.shape[0]
    n = ns + nf + npr

    def coupling(m, k):
        C = sp.random(m, k, density=3.0 / k, random_state=7, format="csr")
        C.data = -0.01 * C.data
        return C
    Csf, Csp, Cfp = coupling(ns, nf), coupling(ns, npr), coupling(nf, npr)
    A = sp.bmat([[Ks, Csf, Csp], [Csf.T, Kf, Cfp], [Csp.T, Cfp.T, Kp]], format="csr")
    A.sort_indices()
    is_s = np.arange(ns, dtype=np.int32)
    is_f = np.arange(ns, ns + nf, dtype=np.int32)
    is_p = np.arange(ns + nf, n, dtype=np.int32)
    return A, is_s, is_f, is_p


def _apply(A, is_s, is_f, is_p, x, extra):
    from lib.handle import Handle, params_to_options
    opts = dict(DB, **extra)
    opts.update(params_to_options(PARAMS))
    h = Handle.from_csr(A, A, None, is_s, is_f, is_p, [], opts)
    y = h.pc_apply(x)
    h.destroy()
    return y


def test_window_sweep_long_block_matches_workgroup_sweep(gpu, capfd):
    A, is_s, is_f, is_p = _system()
    x = np.random.default_rng(3).standard_normal(A.shape[0])
    capfd.readouterr()
    yw = _apply(A, is_s, is_f, is_p, x, {"pls.sweep_window": "1"})
    err = capfd.readouterr().err
    lines = [ln for ln in err.splitlines() if ln.startswith("[pls ilu]")]
    assert any("n 19880 " in ln and "sweep window" in ln for ln in lines), lines
    assert any("n 12300 " in ln and "sweep window" in ln for ln in lines), lines
    yl = _apply(A, is_s, is_f, is_p, x, {"pls.sweep_window": "0", "pls.sweep_chain": "0"})
    err = capfd.readouterr().err
    assert all("sweep lds" in ln for ln in err.splitlines() if ln.startswith("[pls ilu]")), err
    o = OracleSolver(A, A, None, is_s, is_f, is_p, PARAMS, {k: v for k, v in DB.items() if not k.startswith("pls.")}, [])
    yo = o.block_pc.apply(x)
    scale = np.max(np.abs(yo))
    # the window inverses reassociate the sums: 1e-12 as for the other window cases
    assert np.max(np.abs(yw - yo)) <= 1e-12 * scale
    assert np.max(np.abs(yl - yo)) <= 1e-13 * scale
    assert np.max(np.abs(yw - yl)) <= 1e-12 * scale


def _sweeps(err):
    return [ln for ln in err.splitlines() if ln.startswith("[pls ilu]")]


@pytest.mark.parametrize("depth", ["2", "3"])
def test_window_ring_matches_window_sweep(gpu, capfd, depth):
    """The window sweep's ring variant (blocks longer than LDS: y as the block
    solution, an LDS ring of the last 16,384 rows for the off-window terms,
    input rows prefetched from global memory with the window's data) forced on
    the LDS-resident blocks above, with 2 or 3 windows of data in flight: the
    same sums in the same order, so bitwise the LDS variant."""
    A, is_s, is_f, is_p = _system()
    x = np.random.default_rng(3).standard_normal(A.shape[0])
    capfd.readouterr()
    yw = _apply(A, is_s, is_f, is_p, x, {"pls.sweep_window": "1"})
    assert not any("window-ring" in ln for ln in _sweeps(capfd.readouterr().err))
    yr = _apply(A, is_s, is_f, is_p, x, {"pls.sweep_window": "1", "pls.window_ring": "1", "pls.window_depth": depth})
    lines = _sweeps(capfd.readouterr().err)
    assert any("n 19880 " in ln and "sweep window-ring" in ln for ln in lines), lines
    assert np.array_equal(yr, yw)


@pytest.mark.parametrize("ring", ["0", "1"])
def test_window_records_per_wave(gpu, capfd, ring):
    """The window sweep loads 4 stream records per wave and window where no row
    of the triangle has more than 16 off-window entries (these 5-point blocks:
    1), 6 up to 24, else 8 (pls.window_kpw 8 forces 8): the same sums, bitwise."""
    A, is_s, is_f, is_p = _system()
    x = np.random.default_rng(3).standard_normal(A.shape[0])
    capfd.readouterr()
    base = {"pls.sweep_window": "1", "pls.window_ring": ring}
    y4 = _apply(A, is_s, is_f, is_p, x, base)
    assert any("n 19880 " in ln and "(records 4/4)" in ln for ln in _sweeps(capfd.readouterr().err))
    y8 = _apply(A, is_s, is_f, is_p, x, dict(base, **{"pls.window_kpw": "8"}))
    assert any("n 19880 " in ln and "(records 8/8)" in ln for ln in _sweeps(capfd.readouterr().err))
    assert np.array_equal(y4, y8)


@pytest.mark.parametrize("mixed", ["0", "1"])
def test_window_ring_long_block(gpu, capfd, mixed):
    """A 36,000-row block (563 windows, beyond the 19,904-row LDS window): the
    ring variant -- both triangles in windows, or (mixed) L by the y-resident
    level sweep and U in windows -- against the oracle and against the
    one-workgroup GMEM sweep that ran there before (1e-12: the window inverses
    reassociate the sums)."""
    rng = np.random.default_rng(5)
    Ks = _grid_block(200, 180, rng)
    Kf = _grid_block(40, 40, rng)
    Kp = _grid_block(30, 30, rng)
    ns, nf, npr = Ks.shape[0], Kf.shape[0], Kp.shape[0]
    A = sp.block_diag([Ks, Kf, Kp], format="csr")
    A.sort_indices()
    is_s = np.arange(ns, dtype=np.int32)
    is_f = np.arange(ns, ns + nf, dtype=np.int32)
    is_p = np.arange(ns + nf, ns + nf + npr, dtype=np.int32)
    x = np.random.default_rng(4).standard_normal(A.shape[0])
    capfd.readouterr()
    yr = _apply(A, is_s, is_f, is_p, x, {"pls.sweep_window": "1", "pls.window_mixed": mixed})
    lines = _sweeps(capfd.readouterr().err)
    kind = "sweep levels+window-ring" if mixed == "1" else "sweep window-ring"
    assert any("n 36000 " in ln and kind in ln for ln in lines), lines
    yg = _apply(A, is_s, is_f, is_p, x, {"pls.sweep_window": "0", "pls.window_ring": "0"})
    lines = _sweeps(capfd.readouterr().err)
    assert any("n 36000 " in ln and "window" not in ln for ln in lines), lines
    o = OracleSolver(A, A, None, is_s, is_f, is_p, PARAMS, {k: v for k, v in DB.items() if not k.startswith("pls.")}, [])
    yo = o.block_pc.apply(x)
    scale = np.max(np.abs(yo))
    assert np.max(np.abs(yr - yo)) <= 1e-12 * scale
    assert np.max(np.abs(yg - yo)) <= 1e-13 * scale


@pytest.mark.parametrize("N,blocks,variant", [
    (16, 24, {}),
    (16, 24, {"pls.fp_pipeline_depth": "6"}),
    (16, 24, {"pls.fp_pipeline_rr": "2"}),
    (16, 24, {"pls.fp_pipeline_rr": "4"}),
])
def test_fp_pipeline_bitwise(gpu, capfd, N, blocks, variant):
    """The 2-way PC's pressure-first pipeline (pls.fp_pipeline, capi.cpp
    setup_fp_pipeline): the heavy pressure BJACOBI blocks of the fp block get
    their rows of t = x_fp - P_fp,s y_s first and sweep on a second stream.
    Same per-row sums and per-block sweeps as the plain path: PC applies and
    whole solves bitwise equal, and the pipeline must have engaged.  Also the
    experimental heavy-sweep variants: 6 levels in flight on 8
    waves (sweep2_deep) and round-robin wave groups of 2 / 4 (sweep_rr)."""
    from lib.handle import Handle, params_to_options
    from oracle import synthetic as S
    spec = S.SynthSpec(3, N)
    params = dict(PARAMS, **{"solver maxiter": 200})
    db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "s_ksp_type": "preonly", "s_pc_type": "bjacobi",
          "s_pc_bjacobi_blocks": str(blocks), "fp_ksp_type": "preonly", "fp_pc_type": "bjacobi",
          "fp_pc_bjacobi_blocks": str(blocks), "pls.ilu_view": "1"}
    out = {}
    for pipe in ("1", "0"):
        opts = dict(db, **{"pls.fp_pipeline": pipe}, **(variant if pipe == "1" else {}))
        opts.update(params_to_options(params))
        capfd.readouterr()
        h = Handle.synthetic(spec.dim, spec.N, spec.seed, spec.delta, opts)
        x = np.random.default_rng(4).standard_normal(spec.n)
        y = h.pc_apply(x)
        b = S.rhs(spec)
        xs, r = h.solve(b)
        out[pipe] = (y, xs, r.its, r.reason, h.history())
        h.destroy()
        err = capfd.readouterr().err
        assert ("[pls fp pipeline]" in err) == (pipe == "1"), err
    a, b_ = out["1"], out["0"]
    assert np.array_equal(a[0], b_[0])
    assert np.array_equal(a[1], b_[1])
    assert a[2] == b_[2] and a[3] == b_[3]
    assert np.array_equal(a[4], b_[4])


def _fe_apply(s, two_way, extra):
    from lib.handle import Handle, params_to_options
    params = dict(PARAMS, **{"pc type": "diagonal" if two_way else "diagonal 3-way"})
    db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "pls.ilu_view": "1"}
    for pre in (("s_", "fp_") if two_way else ("s_", "f_", "p_", "diff_")):
        db[pre + "ksp_type"] = "preonly"
        db[pre + "pc_type"] = "ilu"
    opts = dict(db, **extra)
    opts.update(params_to_options(params))
    h = Handle.from_csr(s.A, s.P, s.P_diff, s.is_s, s.is_f, s.is_p, s.bcs_sub_pressure, opts)
    x = np.random.default_rng(8).standard_normal(s.A.shape[0])
    y = h.pc_apply(x)
    h.destroy()
    o = OracleSolver(s.A, s.P, s.P_diff, s.is_s, s.is_f, s.is_p, params,
                     {k: v for k, v in db.items() if not k.startswith("pls.")}, s.bcs_sub_pressure)
    return y, o.block_pc.apply(x)


@pytest.mark.parametrize("N,gmem", [(4, "1"), (12, "0")])
def test_swin_sweep_matches_oracle(gpu, capfd, N, gmem):
    """Whole-block ILU(0) on assembled 3-D swelling blocks through the super-
    window sweep (pls.sweep_swin 1: 64-row windows with explicit inverses,
    near terms from LDS, far terms from the block solution in global memory;
    lib/Preconditioner.py:94-100's ILU).  N = 4 with every block forced
    y-resident (pls.ilu_gmem 1), N = 12 at its size (s 46,875 / fp 49,072
    rows, beyond LDS).  Bar: the window inverses reassociate the sums, <= 1e-12
    of max |y| against the oracle; the ring sweep (pls.sweep_swin 0) on the
    same blocks as a second reference."""
    from lib.fe_swelling import assemble_swelling
    s = assemble_swelling(3, N, "diagonal")
    capfd.readouterr()
    ysw, yo = _fe_apply(s, True, {"pls.sweep_swin": "1", "pls.ilu_gmem": gmem})
    err = capfd.readouterr().err
    kinds = [ln for ln in err.splitlines() if ln.startswith("[pls ilu]")]
    assert kinds and all("sweep swin" in ln for ln in kinds), kinds
    yr, _ = _fe_apply(s, True, {"pls.sweep_swin": "0", "pls.ilu_gmem": gmem})
    scale = np.max(np.abs(yo))
    assert np.max(np.abs(ysw - yo)) <= 1e-12 * scale
    assert np.max(np.abs(ysw - yr)) <= 1e-12 * scale


def test_swin_sweep_three_way(gpu, capfd):
    """3-way (FS and DIFF sweeps on two streams share the s / f PCs: the super-
    window sweep must be reentrant) on the 3-D N=4 system, every block forced
    y-resident."""
    from lib.fe_swelling import assemble_swelling
    s = assemble_swelling(3, 4, "diagonal 3-way")
    ysw, yo = _fe_apply(s, False, {"pls.sweep_swin": "1", "pls.ilu_gmem": "1"})
    assert np.max(np.abs(ysw - yo)) <= 1e-12 * np.max(np.abs(yo))
