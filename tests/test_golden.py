"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle reproduces every fixture (regression pin of the oracle).
GPU: libpls.so reproduces every fixture through the C-ABI -- iteration count
and reason exact, residual history within 1e-10 relative (AAR: the attainable
accuracy bound of test_gpu_parity), solution within 1e-8.
"""
import glob
import json
import os

import numpy as np
import pytest

from oracle import synthetic as S

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(glob.glob(os.path.join(HERE, "*.npz")))


def load(path):
    z = np.load(path, allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    return meta, int(z["its"]), int(z["reason"]), z["history"], z["x"]


def spec_of(meta):
    return S.SynthSpec(meta["dim"], meta["N"], meta["seed"], meta["delta"])


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[:-4] for f in FILES])
def test_oracle_reproduces_golden(path):
    from oracle.solver import OracleSolver
    meta, its, reason, hist, x = load(path)
    spec = spec_of(meta)
    A, P, Pd = S.matrix(spec, 0), S.matrix(spec, 1), S.matrix(spec, 2)
    is_s, is_f, is_p = S.field_major_index_sets(spec)
    o = OracleSolver(A, P, Pd, is_s, is_f, is_p, meta["params"], meta["db"], S.bcs_sub_pressure(spec))
    xo = o.solve(S.rhs(spec))
    assert o.its == its and o.reason == reason
    assert np.allclose(o.history, hist, rtol=1e-12, atol=0)
    assert np.allclose(xo, x, rtol=1e-12, atol=1e-14)


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[:-4] for f in FILES])
def test_device_reproduces_golden(gpu, path):
    from lib.handle import Handle, params_to_options
    meta, its, reason, hist, x = load(path)
    spec = spec_of(meta)
    opts = dict(meta["db"])
    opts.update(params_to_options(meta["params"]))
    h = Handle.synthetic(spec.dim, spec.N, spec.seed, spec.delta, opts)
    xd, r = h.solve(S.rhs(spec))
    hd = h.history()
    assert r.its == its and r.reason == reason
    if meta["params"]["solver type"] == "aar":
        bound = 1e-10 * np.abs(hist) + 100 * np.finfo(float).eps * hist[0]
        assert np.all(np.abs(hd - hist) <= bound)
    else:
        assert np.max(np.abs(hd - hist) / np.abs(hist)) <= 1e-10
    assert np.linalg.norm(xd - x) <= 1e-8 * np.linalg.norm(x)
