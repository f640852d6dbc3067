"""Standalone AndersonAcceleration (reference lib/AndersonAcceleration.py:6-78)
through pls_anderson_* against the oracle's restatement (oracle/aar.py).

The same sequence of g_k vectors goes to both (open loop: the oracle's own
fixed-point iteration x_{k+1} = G(x_k) generates it), so each mixed iterate is
compared without feedback.  Bound: relative to ||x_k||, 10x the oracle's own
deviation when its numpy QR is swapped for the device's TSQR (measured per
case), at least 1e-11 (the open loop carries the device's rounding through up
to 24 steps of X / F histories: 1.7e-12 measured at step 20 of n = 1000,
order 3); cond(R) recorded by the oracle and asserted small.  The g_k repeated twice in a row
exercises the reference's ||delta f|| < 1e-12 branch (AndersonAcceleration.py:
44-46: k -= 1, x_k = g_k)."""
import numpy as np
import pytest

from oracle.aar import AndersonAcceleration as OracleAA

pytestmark = pytest.mark.gpu


def _sequence(n, order, steps, seed, lstsq=None):
    """g_k of a damped linear fixed-point map mixed by the oracle (lstsq: the
    oracle's least-squares hook, e.g. the device's TSQR algorithm)."""
    rng = np.random.default_rng(seed)
    M = rng.standard_normal((n, n)) / np.sqrt(n)
    M = 0.9 * M / np.max(np.abs(np.linalg.eigvals(M)))
    c = rng.standard_normal(n)
    aa = OracleAA(order)
    aa.lstsq = lstsq
    x = np.zeros(n)
    gs, xs = [], []
    for k in range(steps):
        g = M @ x + c
        if k == 4:  # a repeated g: delta f == 0 on the next call
            gs.append(g.copy())
            xs.append(aa.get_next_vector(g.copy()))
        gs.append(g.copy())
        x = aa.get_next_vector(g.copy())
        xs.append(x.copy())
    return gs, xs, aa.max_cond


@pytest.mark.parametrize("n,order,steps", [(300, 1, 24), (1000, 3, 24), (2048, 5, 24), (4096, 10, 10)])
def test_anderson_matches_oracle(gpu, n, order, steps):
    from lib.AndersonAcceleration import AndersonAcceleration
    from oracle.aar import tsqr_lstsq
    gs, xs, cond = _sequence(n, order, steps, seed=n + order)
    assert cond < 1e8
    # bound: 10x the oracle's own deviation when its numpy QR is replaced by the
    # device's Householder TSQR (same g sequence), at least 1e-12
    _, xt, _ = _sequence(n, order, steps, seed=n + order, lstsq=tsqr_lstsq)
    tol = max(1e-11, 10 * max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(xt, xs)))
    aa = AndersonAcceleration(order)
    try:
        for k, (g, xo) in enumerate(zip(gs, xs)):
            v = g.copy()
            out = aa.get_next_vector(v)
            assert out is v  # in place, as the reference's self.xk.copy(gk)
            err = np.linalg.norm(v - xo) / np.linalg.norm(xo)
            assert err <= tol, (k, err, tol)
    finally:
        aa.destroy()


def test_anderson_device_vector_and_order0(gpu):
    """A DeviceArray is mixed on the device in place; order 0 is the identity
    (mk = 0 on every call: x_k = g_k)."""
    import lib._native as N
    from lib.AndersonAcceleration import AndersonAcceleration
    gs, xs, _ = _sequence(512, 2, 10, seed=5)
    aa = AndersonAcceleration(2)
    d = N.DeviceArray(512)
    try:
        for g, xo in zip(gs, xs):
            d.upload(g)
            aa.get_next_vector(d)
            assert np.linalg.norm(d.download() - xo) <= 1e-12 * np.linalg.norm(xo)
        with pytest.raises(ValueError):
            aa.get_next_vector(np.zeros(3))
    finally:
        d.free()
        aa.destroy()
    a0 = AndersonAcceleration(0)
    g = np.random.default_rng(1).standard_normal(64)
    for _ in range(3):
        v = g.copy()
        assert np.array_equal(a0.get_next_vector(v), g)
    a0.destroy()
