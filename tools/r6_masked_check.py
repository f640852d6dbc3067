"""Bitwise check of the ring window sweep's masked-load variant (pls.ring_probe
65536, experimental) against the default, on the 36,000-row block of
tests/test_gpu_sweeps.py (run on the GPU box)."""
import os
import sys

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "poroelasticity-linear-solvers_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import test_gpu_sweeps as T  # noqa: E402

rng = np.random.default_rng(5)
Ks, Kf, Kp = T._grid_block(200, 180, rng), T._grid_block(40, 40, rng), T._grid_block(30, 30, rng)
ns, nf, npr = Ks.shape[0], Kf.shape[0], Kp.shape[0]
A = sp.block_diag([Ks, Kf, Kp], format="csr")
A.sort_indices()
is_s = np.arange(ns, dtype=np.int32)
is_f = np.arange(ns, ns + nf, dtype=np.int32)
is_p = np.arange(ns + nf, ns + nf + npr, dtype=np.int32)
x = np.random.default_rng(4).standard_normal(A.shape[0])
for mixed in ("0", "1"):
    y0 = T._apply(A, is_s, is_f, is_p, x, {"pls.sweep_window": "1", "pls.window_mixed": mixed})
    y1 = T._apply(A, is_s, is_f, is_p, x, {"pls.sweep_window": "1", "pls.window_mixed": mixed, "pls.ring_probe": "65536"})
    print("mixed", mixed, "bitwise" if np.array_equal(y0, y1) else f"DIFF {np.max(np.abs(y0 - y1))}", flush=True)
