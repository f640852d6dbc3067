"""Compare tools/g8_n27.py's GPU histories with OracleSolver(dist_size=G)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "poroelasticity-linear-solvers_amd")):
    sys.path.insert(0, p)
from oracle import synthetic as S  # noqa: E402
from oracle.solver import OracleSolver  # noqa: E402

G, N = int(sys.argv[1]), int(sys.argv[2])
d = os.path.join(ROOT, "gpurun_out", "r5", f"g{G}n{N}")
c = json.load(open(os.path.join(d, "case.json")))
parts = [dict(np.load(os.path.join(d, f"{c['name']}_rank{r}.npz"))) for r in range(G)]
spec = S.SynthSpec(3, N)
A, P, Pd = S.matrix(spec, 0), S.matrix(spec, 1), S.matrix(spec, 2)
is_s, is_f, is_p = S.field_major_index_sets(spec)
t = time.time()
o = OracleSolver(A, P, Pd, is_s, is_f, is_p, c["params"], c["db"], S.bcs_sub_pressure(spec), dist_size=G)
o.solve(S.rhs(spec))
ho = np.asarray(o.history)
h = parts[0]["hist"]
m = min(len(h), len(ho))
print(f"oracle its {o.its} reason {o.reason} ({time.time() - t:.0f} s); device its {int(parts[0]['its'])} "
      f"reason {int(parts[0]['reason'])}; max history rel diff {np.max(np.abs(h[:m] - ho[:m]) / ho[:m]):.2e}")
