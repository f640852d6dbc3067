"""Headline configuration (BASELINE.json configs[1]) against the oracle at its
full size.

The metric point (3-D N=59, 10.33M DoF, 1.88 G nnz), the size configs[1]
names (N=64, 13.15M DoF) and the "~1M DoF" point (N=27) are solved twice on the same system -- by libpls on the GPU and by the
oracle's C/OpenMP restatement of the identical algorithm
(``oracle/csrc/cpu_solver.c``: right-PC GMRES, CGS, Givens, BuildSoln with the
extra PC apply, the 2-way PC of reference ``lib/Preconditioner.py:219-246``,
PREONLY + BJACOBI(ILU(0)) blocks with PETSc's block sizing; itself checked
against the Python oracle in ``tests/test_oracle.py``) -- on the host cores of
the GPU box.  Bar (north_star): iteration count and converged reason exact,
every residual-history entry within 1e-10 relative; the solutions agree to
the accuracy the solve attains (rtol 1e-6 of the GMRES residual).

The host matrices come from the oracle's C generator (``oracle.c``); the
device generates its own copy in HBM (``k_synth_*``), bitwise the same by
construction (``tests/test_gpu_parity.py::test_synthetic_generator_bitwise``), so the two
solvers see identical inputs.  Host memory: A + P at N=59 ~ 45 GB, the CPU
Krylov basis 8.3 GB.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED, DELTA = 20261015, 0.05


def _threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))  # the GPU box's CPU share


# N=64 is configs[1]'s named size (13.15M DoF; 320 / 330 blocks keep every
# block solution in one CU's LDS); host A + P ~ 58 GB, inside the box's cap
@pytest.mark.parametrize("N,nb_s,nb_fp", [(27, 64, 64), (59, 256, 264), (64, 320, 330)])
def test_headline_vs_oracle_full_size(gpu, N, nb_s, nb_fp):
    import lib._native as Nt
    from lib.handle import Handle
    from oracle import native
    from oracle import synthetic as S
    from test_gpu_large import _opts

    spec = S.SynthSpec(3, N, SEED, DELTA)
    ns = spec.sizes()[0]
    b = np.random.default_rng(7).uniform(-1.0, 1.0, spec.n)

    # device first (frees HBM before the host allocations grow)
    h = Handle.synthetic(3, N, SEED, DELTA, _opts(nb_s, nb_fp))
    n = h.n
    assert n == spec.n
    d_b, d_x = Nt.DeviceArray(n), Nt.DeviceArray(n)
    d_b.upload(b)
    res = h.solve_device(d_b.p, d_x.p)
    hist = np.asarray(h.history())
    x = d_x.download()
    d_b.free()
    d_x.free()
    h.destroy()

    A = S.matrix(spec, S.VARIANT_A)
    P = S.matrix(spec, S.VARIANT_P)
    xo, its, reason, ho, _, _ = native.cpu_gmres_2way(A, P, ns, nb_s, nb_fp, b, rtol=1e-6, atol=1e-8, maxit=100,
                                                      nthreads=_threads())
    del A, P

    assert res.its == its, (res.its, its)
    assert res.reason == reason == 2, (res.reason, reason)
    rel = np.abs(hist - ho) / np.abs(ho)
    assert rel.max() <= 1e-10, f"history max rel diff {rel.max():.3e} at entry {int(rel.argmax())}"
    # both solutions carry GMRES's own error (rtol 1e-6 of ||b||); they agree far
    # better than that since the two runs differ only in summation order
    assert np.linalg.norm(x - xo) <= 1e-8 * np.linalg.norm(xo)
