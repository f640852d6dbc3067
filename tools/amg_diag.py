"""Diagnostics: device AMG hierarchy (pls.amg_view) vs the oracle's, per block."""
import sys
sys.path[:0] = ["/root/repo", "/root/repo/tests", "/root/repo/poroelasticity-linear-solvers_amd"]
import numpy as np
from oracle import synthetic as S
import test_gpu_amg as T
from test_gpu_parity import BASE, _handle, _oracle

dim, N = int(sys.argv[1]), int(sys.argv[2])
spec = S.SynthSpec(dim, N)
params = dict(BASE, **{"pc type": "diagonal 3-way", "inner pc type": "lu"})
db = T._amg_db("gamg", {"pls.amg_view": None})
o = _oracle(spec, params, db)
for k in ("ksp_s", "ksp_f", "ksp_p", "ksp_pd"):
    ksp = getattr(o.block_pc, k, None)
    if ksp is None or not hasattr(ksp.pc, "levels"):
        continue
    pc = ksp.pc
    print("oracle", k, [(L["A"].shape[0], L["A"].nnz, repr(L["lam"])) for L in pc.levels], "coarse", pc.coarse.shape[0],
          "Pnnz", [L["P"].nnz for L in pc.levels], flush=True)
h = _handle(spec, params, db)
x = np.random.default_rng(3).standard_normal(spec.n)
y = h.pc_apply(x)
yo = o.block_pc.apply(x)
ns, nf = len(S.field_major_index_sets(spec)[0]), len(S.field_major_index_sets(spec)[1])
for name, sl in (("s", slice(0, ns)), ("f", slice(ns, ns + nf)), ("p", slice(ns + nf, None))):
    print(name, "max rel diff", np.max(np.abs(y[sl] - yo[sl])) / np.max(np.abs(yo[sl])), flush=True)
