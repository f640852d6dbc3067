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
    return G, launch("gpu", CASES, G, str(tmp_path_factory.mktemp(f"dist{G}")), timeout=900)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_dist_solve(ranks, case):
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
    assert np.linalg.norm(Mv - Mo) <= 1e-13 * np.linalg.norm(Mo) * max(1, G)
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
