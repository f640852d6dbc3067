"""Distributed libpls.so (G ranks, one process each) against the oracle.

The G ranks share the box's one GPU and talk through the host-staged
communicator (lib/dist.py ``Communicator.gloo``; RCCL itself refuses two ranks
on one device -- the RCCL backend is exercised at world size 1 below and by
bench.py on multi-GPU nodes).  The kernels, halo plan, ghost remap and
rank-ordered global sums are the same code for both backends.

Reference point: ``OracleSolver(dist_size=G)`` -- the single-process oracle
with the G-rank block-Jacobi structure (oracle/dist.py), itself checked against
a G-process numpy emulation in tests/test_dist_cpu.py.  Tolerances as in
tests/test_gpu_parity.py: synthetic rhs bitwise; SpMV / PC apply <= 1e-13
relative; iteration count and reason exact; history h_k within
1e-10 h_k + 100 eps h_0 (AAR: the measured least-squares noise floor of test_gpu_parity).
"""
import numpy as np
import pytest

from distutil import assemble, launch
from oracle import synthetic as S
from oracle.solver import OracleSolver

pytestmark = pytest.mark.gpu
EPS = np.finfo(np.float64).eps

BASE = {"solver type": "gmres", "solver atol": 1e-10, "solver rtol": 1e-8, "solver maxiter": 300,
        "pc type": "diagonal", "inner ksp type": "preonly", "inner pc type": "ilu", "inner rtol": 1e-6,
        "inner atol": 0, "inner maxiter": 1000, "inner monitor": False, "solver monitor": False,
        "inner accel order": 0, "AAR order": 10, "AAR p": 5, "AAR omega": 1, "AAR beta": 1}


def _db(blocks=None):
    db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right"}
    blocks = blocks or {"s_": 5, "f_": 3, "p_": 2, "diff_": 2, "fp_": 3}
    for pre, nb in blocks.items():
        db[pre + "ksp_type"] = "preonly"
        db[pre + "pc_type"] = "bjacobi"
        db[pre + "pc_bjacobi_blocks"] = str(nb)
    return db


CASES = [
    {"name": "twoway_2d", "dim": 2, "N": 12, "params": BASE, "db": _db()},
    {"name": "threeway_2d", "dim": 2, "N": 10, "params": dict(BASE, **{"pc type": "diagonal 3-way"}), "db": _db()},
    {"name": "twoway_3d", "dim": 3, "N": 4, "params": BASE, "db": _db({"s_": 4, "fp_": 4})},
    # the SpMV layout with 8 segment bases per lane (what the halo rows of large
    # sharded systems need: own s/f/p + a neighbour's s/f/p), forced here
    {"name": "twoway_3d_seg8", "dim": 3, "N": 4, "params": BASE,
     "db": dict(_db({"s_": 4, "fp_": 4}), **{"pls.d16_segs": "8"})},
    {"name": "aar_2d", "dim": 2, "N": 10, "params": dict(BASE, **{"solver type": "aar", "solver maxiter": 200}),
     "db": _db()},
    # configs[4]: AAR depth m=5, p=5 on a 3-D system, sharded
    {"name": "aar_m5_3d", "dim": 3, "N": 4,
     "params": dict(BASE, **{"solver type": "aar", "solver maxiter": 200, "AAR order": 5, "AAR p": 5}),
     "db": _db({"s_": 4, "fp_": 4})},
    {"name": "jacobi_left_2d", "dim": 2, "N": 9, "params": BASE,
     "db": {"global_ksp_type": "gmres", "s_ksp_type": "preonly", "s_pc_type": "jacobi",
            "fp_ksp_type": "preonly", "fp_pc_type": "jacobi"}},
    # whole-block PCs on sharded blocks (PETSc PCREDUNDANT semantics: every rank
    # gathers the block and applies the one-rank PC): ILU(0) and LU ...
    {"name": "redundant_ilu_lu_3way_2d", "dim": 2, "N": 10, "params": dict(BASE, **{"pc type": "diagonal 3-way"}),
     "db": {"global_ksp_type": "gmres", "global_ksp_pc_side": "right",
            "s_ksp_type": "preonly", "s_pc_type": "ilu", "f_ksp_type": "preonly", "f_pc_type": "lu",
            "p_ksp_type": "preonly", "p_pc_type": "lu", "diff_ksp_type": "preonly", "diff_pc_type": "ilu",
            "pls.redundant_ilu": "1"}},
    # ... the classical AMG with petsc-options-inexact's BoomerAMG settings ...
    {"name": "redundant_hypre_3way_3d", "dim": 3, "N": 4, "params": dict(BASE, **{"pc type": "diagonal 3-way"}),
     "pc_tol": 1e-12, "db": dict({"global_ksp_type": "gmres", "global_ksp_pc_side": "right"},
                                 **{pre + k: v for pre in ("s_", "f_", "p_", "diff_") for k, v in {
                                     "ksp_type": "preonly", "pc_type": "hypre", "pc_hypre_boomeramg_P_max": "4",
                                     "pc_hypre_boomeramg_agg_nl": "1", "pc_hypre_boomeramg_agg_num_paths": "2",
                                     "pc_hypre_boomeramg_no_CF": "true"}.items()})},
    # (round 3: hypre on a sharded block runs BoomerAMG's np = G hierarchy with
    # every rank smoothing only its own rows -- the case above -- and with C/F
    # relaxation; the gathered, redundantly applied one stays on request)
    {"name": "dist_hypre_cf_3way_3d", "dim": 3, "N": 4, "params": dict(BASE, **{"pc type": "diagonal 3-way"}),
     "pc_tol": 1e-12, "db": dict({"global_ksp_type": "gmres", "global_ksp_pc_side": "right"},
                                 **{pre + k: v for pre in ("s_", "f_", "p_", "diff_") for k, v in {
                                     "ksp_type": "preonly", "pc_type": "hypre", "pc_hypre_boomeramg_P_max": "4",
                                     "pc_hypre_boomeramg_agg_nl": "1", "pc_hypre_boomeramg_agg_num_paths": "2",
                                     }.items()})},
    {"name": "redundant_hypre_forced_3way_3d", "dim": 3, "N": 4, "params": dict(BASE, **{"pc type": "diagonal 3-way"}),
     "pc_tol": 1e-12, "db": dict({"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "pls.hypre_dist": "0"},
                                 **{pre + k: v for pre in ("s_", "f_", "p_", "diff_") for k, v in {
                                     "ksp_type": "preonly", "pc_type": "hypre", "pc_hypre_boomeramg_P_max": "4",
                                     "pc_hypre_boomeramg_agg_nl": "1", "pc_hypre_boomeramg_agg_num_paths": "2",
                                     "pc_hypre_boomeramg_no_CF": "true"}.items()})},
    # ... and the fp block's Schur fieldsplit (petsc-options-inexact:73-114 with LU splits)
    {"name": "redundant_fieldsplit_2d", "dim": 2, "N": 10, "params": BASE,
     "db": dict(_db({"s_": 5}), **{"fp_ksp_type": "preonly", "fp_pc_type": "fieldsplit",
                                   "fp_pc_fieldsplit_type": "schur", "fp_pc_fieldsplit_schur_fact_type": "lower",
                                   "fp_pc_fieldsplit_schur_precondition": "selfp",
                                   "fp_fieldsplit_0_ksp_type": "preonly", "fp_fieldsplit_0_pc_type": "lu",
                                   "fp_fieldsplit_1_ksp_type": "preonly", "fp_fieldsplit_1_pc_type": "lu"})},
]


def _fe_db(G):
    db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right"}
    for pre in ("s_", "f_", "p_", "diff_", "fp_"):
        db[pre + "ksp_type"] = "preonly"
        db[pre + "pc_type"] = "bjacobi"
        db[pre + "pc_bjacobi_blocks"] = "3"
    return db


# caller-assembled swelling systems (lib/fe_swelling.py, dolfin-like interleaved
# numbering) handed over rank by rank through pls_create_dist: every rank
# passes its PETSc-split rows (global columns) and the index sets of the dofs
# it owns -- the reference's mpirun path (paper-scripts/robustness_2d.sh:29)
def _fs_db():
    db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "s_ksp_type": "preonly", "s_pc_type": "bjacobi",
          "s_pc_bjacobi_blocks": "3", "fp_ksp_type": "preonly", "fp_pc_type": "fieldsplit",
          "fp_pc_fieldsplit_type": "schur", "fp_pc_fieldsplit_schur_fact_type": "lower",
          "fp_pc_fieldsplit_schur_precondition": "selfp"}
    db.update({"fp_fieldsplit_0_ksp_type": "preonly", "fp_fieldsplit_0_pc_type": "ilu",
               "fp_fieldsplit_1_ksp_type": "preonly", "fp_fieldsplit_1_pc_type": "lu"})
    return db


FE_BASE = dict(BASE, **{"solver atol": 1e-8, "solver rtol": 1e-6, "solver maxiter": 60, "inner pc type": "bjacobi"})
FE_CASES = [
    {"name": "fe_threeway_2d", "system": "fe", "dim": 2, "N": 8,
     "params": dict(FE_BASE, **{"pc type": "diagonal 3-way"}), "db": _fe_db(3)},
    {"name": "fe_threeway_3d", "system": "fe", "dim": 3, "N": 3,
     "params": dict(FE_BASE, **{"pc type": "diagonal 3-way"}), "db": _fe_db(3)},
    {"name": "fe_twoway_3d", "system": "fe", "dim": 3, "N": 3,
     "params": dict(FE_BASE, **{"pc type": "diagonal"}), "db": _fe_db(3)},
    # the same through the unchanged facade call sequence (lib/Preconditioner.py,
    # lib/Solver.py inside a torch.distributed job)
    {"name": "fe_facade_threeway_2d", "system": "fe", "facade": True, "dim": 2, "N": 8,
     "params": dict(FE_BASE, **{"pc type": "diagonal 3-way"}), "db": _fe_db(3)},
    {"name": "fe_facade_twoway_3d", "system": "fe", "facade": True, "dim": 3, "N": 3,
     "params": dict(FE_BASE, **{"pc type": "diagonal"}), "db": _fe_db(3)},
    # 2-way with a Schur fieldsplit on the fp block (petsc-options-inexact's fp_
    # structure, linear split solves): under pls_create_dist every rank's fp rows
    # interleave f and p, so the gathered block's splits come from every rank's
    # fp index sets (they were taken as field-major slabs)
    {"name": "fe_fieldsplit_twoway_2d", "system": "fe", "dim": 2, "N": 8,
     "params": dict(FE_BASE, **{"pc type": "diagonal", "solver maxiter": 200}), "db": _fs_db()},
    {"name": "fe_facade_fieldsplit_twoway_2d", "system": "fe", "facade": True, "dim": 2, "N": 8,
     "params": dict(FE_BASE, **{"pc type": "diagonal", "solver maxiter": 200}), "db": _fs_db()},
    # petsc-options-inexact's BoomerAMG on every block of a caller-assembled
    # system under mpirun: hypre's np = G hierarchy, each rank its own rows
    {"name": "fe_hypre_threeway_2d", "system": "fe", "dim": 2, "N": 8,
     "params": dict(FE_BASE, **{"pc type": "diagonal 3-way", "inner pc type": "hypre", "solver maxiter": 200}),
     "db": dict({"global_ksp_type": "gmres", "global_ksp_pc_side": "right"},
                **{pre + k: v for pre in ("s_", "f_", "p_", "diff_") for k, v in {
                    "ksp_type": "preonly", "pc_type": "hypre", "pc_hypre_boomeramg_P_max": "4",
                    "pc_hypre_boomeramg_agg_nl": "1", "pc_hypre_boomeramg_agg_num_paths": "2",
                    "pc_hypre_boomeramg_no_CF": "true"}.items()})},
    # the reference's exact option set under mpirun (MUMPS LU on every block ->
    # each sharded block gathered and factored redundantly)
    {"name": "fe_exact_lu_threeway_2d", "system": "fe", "dim": 2, "N": 8,
     "params": dict(FE_BASE, **{"pc type": "diagonal 3-way", "inner pc type": "lu"}),
     "db": dict({"global_ksp_type": "gmres", "global_ksp_pc_side": "right"},
                **{pre + k: v for pre in ("s_", "f_", "p_", "diff_") for k, v in
                   (("ksp_type", "preonly"), ("pc_type", "lu"))})},
]


# G = 4 and 8 ranks (the north star's bar is its-exact at 8 GPUs;
# paper-scripts/robustness_2d.sh:9,29 runs mpirun -np 8): BJACOBI 2-way,
# BoomerAMG's np = G hierarchy (C/F relaxation, 3-way), AAR m = 5, and the
# bench's --inner hypre shape (BoomerAMG on the s block, BJACOBI on fp) at
# 3-D N = 10, whose coarsest levels leave ranks without rows
_HYPRE_INEXACT = {"ksp_type": "preonly", "pc_type": "hypre", "pc_hypre_boomeramg_P_max": "4",
                  "pc_hypre_boomeramg_agg_nl": "1", "pc_hypre_boomeramg_agg_num_paths": "2"}
BIG_CASES = [
    {"name": "big_twoway_3d", "dim": 3, "N": 6, "params": BASE, "db": _db({"s_": 8, "fp_": 8})},
    {"name": "big_hypre_cf_3way_3d", "dim": 3, "N": 4, "params": dict(BASE, **{"pc type": "diagonal 3-way"}),
     "pc_tol": 1e-12, "db": dict({"global_ksp_type": "gmres", "global_ksp_pc_side": "right"},
                                 **{pre + k: v for pre in ("s_", "f_", "p_", "diff_") for k, v in _HYPRE_INEXACT.items()})},
    {"name": "big_aar_m5_3d", "dim": 3, "N": 6,
     "params": dict(BASE, **{"solver type": "aar", "solver maxiter": 200, "AAR order": 5, "AAR p": 5}),
     "db": _db({"s_": 8, "fp_": 8})},
    {"name": "big_hypre_s_bjacobi_fp_3d", "dim": 3, "N": 10, "pc_tol": 1e-12,
     "params": dict(BASE, **{"solver rtol": 1e-6, "solver atol": 1e-8}),
     "db": dict({"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "fp_ksp_type": "preonly",
                 "fp_pc_type": "bjacobi", "fp_pc_bjacobi_blocks": "16"},
                **{"s_" + k: v for k, v in dict(_HYPRE_INEXACT, pc_hypre_boomeramg_no_CF="true").items()})},
]


def _oracle(case, G):
    spec = S.SynthSpec(case["dim"], case["N"])
    A, P, Pd = S.matrix(spec, 0), S.matrix(spec, 1), S.matrix(spec, 2)
    is_s, is_f, is_p = S.field_major_index_sets(spec)
    o = OracleSolver(A, P, Pd, is_s, is_f, is_p, case["params"], case["db"], S.bcs_sub_pressure(spec),
                     dist_size=G)
    return spec, A, o


@pytest.fixture(scope="module", params=[2, 3])
def ranks(request, tmp_path_factory):
    G = request.param
    return G, launch("gpu", CASES + FE_CASES, G, str(tmp_path_factory.mktemp(f"dist{G}")), timeout=900)


@pytest.fixture(scope="module", params=[4, 8])
def ranks_big(request, tmp_path_factory):
    G = request.param
    return G, launch("gpu", BIG_CASES, G, str(tmp_path_factory.mktemp(f"distbig{G}")), timeout=900)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_dist_solve(ranks, case):
    _check_dist_solve(ranks, case)


@pytest.mark.parametrize("case", BIG_CASES, ids=[c["name"] for c in BIG_CASES])
def test_dist_solve_g4_g8(ranks_big, case):
    _check_dist_solve(ranks_big, case)


def _check_dist_solve(ranks, case):
    G, res = ranks
    parts = res[case["name"]]
    spec, A, o = _oracle(case, G)
    b = S.rhs(spec)
    # device-generated rhs of each rank's rows: bitwise
    for p in parts:
        assert np.array_equal(p["b_dev"], p["b"])
    # SpMV with halo exchange
    v = parts[0]["v"]
    Av = assemble(parts, "Av")
    ref = A @ v
    assert np.max(np.abs(Av - ref) / (abs(A) @ np.abs(v))) <= 1e-13
    # one PC application (G-rank block structure)
    Mv = assemble(parts, "Mv")
    Mo = o.block_pc.apply(v)
    assert np.linalg.norm(Mv - Mo) <= case.get("pc_tol", 1e-13) * np.linalg.norm(Mo) * max(1, G)
    # the solve
    xo = o.solve(b)
    ho = np.asarray(o.history)
    cond = getattr(o.solver, "max_cond", 1.0)
    tol = 1e-10
    if cond > 1.0:
        # measured noise floor of the Anderson least squares (test_gpu_parity):
        # the oracle's history with numpy QR swapped for the device's TSQR
        from oracle.aar import tsqr_lstsq
        _, _, o2 = _oracle(case, G)
        o2.solver.lstsq = tsqr_lstsq
        o2.solve(b)
        h2 = np.asarray(o2.history)
        m = min(len(h2), len(ho))
        tol = max(tol, 10 * float(np.max(np.abs(h2[:m] - ho[:m]) / (np.abs(ho[:m]) + 100 * EPS * ho[0]))))
    for p in parts:
        assert int(p["its"]) == o.its, (int(p["its"]), o.its)
        assert int(p["reason"]) == o.reason
        h = p["hist"]
        assert h.shape == ho.shape
        worst = np.max(np.abs(h - ho) / (tol * ho + 100 * EPS * ho[0]))
        assert worst <= 1.0, f"history off by {worst:.2f}x the bound"
    x = assemble(parts)
    assert np.linalg.norm(x - xo) <= max(1e-8, tol) * np.linalg.norm(xo)


@pytest.mark.parametrize("case", FE_CASES, ids=[c["name"] for c in FE_CASES])
def test_dist_fe_caller_matrices(ranks, case):
    """pls_create_dist vs OracleSolver(dist_owner=...): the G-rank block
    Jacobi of a caller-assembled system splits every field block by the rows
    each rank owns.  Bar: SpMV / PC apply <= 1e-13; its and reason exact;
    history within max(1e-10, 10x the oracle's own deviation under 1e-15
    relative perturbations of its inner PC outputs) -- these saddle-point
    systems amplify rounding (tests/test_gpu_fe.py)."""
    from lib import fe_swelling as F
    from oracle.dist import row_owner
    G, res = ranks
    parts = res[case["name"]]
    s = F.assemble_swelling(case["dim"], case["N"], case["params"]["pc type"], ordering="interleaved")
    n = s.A.shape[0]
    v = parts[0]["v"]
    Av = assemble(parts, "Av")
    assert np.max(np.abs(Av - s.A @ v) / (abs(s.A) @ np.abs(v) + 1e-300)) <= 1e-13

    def oracle():
        return OracleSolver(s.A, s.P, s.P_diff, s.is_s, s.is_f, s.is_p, case["params"], case["db"],
                            s.bcs_sub_pressure, dist_owner=row_owner(n, G))

    o = oracle()
    Mv = assemble(parts, "Mv")
    Mo = o.block_pc.apply(v)
    assert np.linalg.norm(Mv - Mo) <= 1e-13 * np.linalg.norm(Mo) * G
    xo = o.solve(s.b)
    ho = np.asarray(o.history)
    # noise floor: the oracle's own history under 1e-15 perturbations of its inner PC outputs
    worst = 0.0
    for seed in range(3):
        o2 = oracle()
        rng = np.random.default_rng(seed)
        for name in ("ksp_s", "ksp_fp", "ksp_f", "ksp_p", "ksp_p_diff"):
            ksp = getattr(o2.block_pc, name, None)
            if ksp is not None:
                f = ksp.pc.apply
                ksp.pc.apply = (lambda f: lambda x: (lambda y: y * (1 + 1e-15 * rng.standard_normal(y.size)))(f(x)))(f)
        o2.solve(s.b)
        h2 = np.asarray(o2.history)
        m = min(len(h2), len(ho))
        worst = max(worst, float(np.max(np.abs(h2[:m] - ho[:m]) / np.abs(ho[:m]))))
    tol = max(1e-10, 10 * worst)
    for p in parts:
        assert int(p["its"]) == o.its and int(p["reason"]) == o.reason, (int(p["its"]), o.its)
        h = p["hist"]
        assert h.shape == ho.shape
        assert np.max(np.abs(h - ho) / np.abs(ho)) <= tol
    x = assemble(parts)
    assert np.linalg.norm(x - xo) <= max(1e-8, tol) * np.linalg.norm(xo)


def test_rccl_world1(gpu):
    """RCCL communicator at world size 1 (ncclCommInitRank on this GPU) gives
    the serial handle's result bitwise."""
    import ctypes as C
    import lib._native as N
    from lib.dist import Communicator
    from lib.handle import Handle, params_to_options
    buf = C.create_string_buffer(128)
    N.check(N.lib().pls_rccl_unique_id(buf))
    out = C.c_void_p()
    N.check(N.lib().pls_comm_create_rccl(buf, 0, 1, C.byref(out)))
    comm = Communicator(out, 0, 1)
    case = CASES[0]
    spec = S.SynthSpec(case["dim"], case["N"])
    opts = dict(case["db"])
    opts.update(params_to_options(case["params"]))
    hd = Handle.synthetic_dist(spec.dim, spec.N, spec.seed, spec.delta, opts, comm)
    hs = Handle.synthetic(spec.dim, spec.N, spec.seed, spec.delta, opts)
    b = S.rhs(spec)
    xd, rd = hd.solve(b)
    xs, rs = hs.solve(b)
    assert rd.its == rs.its and np.array_equal(xd, xs)
    hd.destroy()
    comm.destroy()
