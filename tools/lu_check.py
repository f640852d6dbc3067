"""Diagnostics: ||M y - x|| / ||x|| of the 2-way 'diagonal' block PC with PREONLY + LU
on every block (M = P with its s-fp block zeroed) for a chosen LU path, on the
synthetic system and the assembled footing system."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poroelasticity-linear-solvers_amd")]
import numpy as np  # noqa: E402

import lib._native as Nat  # noqa: E402
from lib.handle import Handle, params_to_options  # noqa: E402

BASE = {"solver type": "gmres", "solver atol": 1e-10, "solver rtol": 1e-8, "solver maxiter": 300,
        "pc type": "diagonal", "inner ksp type": "preonly", "inner pc type": "lu", "inner accel order": 0,
        "AAR order": 10, "AAR p": 5, "AAR omega": 1, "AAR beta": 1}


def check(name, A, P, is_s, is_f, is_p, extra):
    db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right"}
    for pre in ("s_", "fp_"):
        db[pre + "ksp_type"] = "preonly"
        db[pre + "pc_type"] = "lu"
    db.update(extra)
    opts = dict(db)
    opts.update(params_to_options(BASE))
    h = Handle.from_csr(A, P, None, is_s, is_f, is_p, [], opts)
    x = np.random.default_rng(3).standard_normal(A.shape[0])
    y = h.pc_apply(x)
    M = P.tolil()
    fp = np.concatenate([is_f, is_p])
    Mc = P.tocsr().copy()
    mask = np.zeros(A.shape[0], bool)
    mask[is_s] = True
    coo = Mc.tocoo()
    keep = ~(mask[coo.row] & ~mask[coo.col])  # drop rows in s, columns in fp
    Mb = type(Mc)((coo.data[keep], (coo.row[keep], coo.col[keep])), shape=Mc.shape).tocsr()
    rs = np.linalg.norm((Mb @ y - x)[is_s]) / np.linalg.norm(x[is_s])
    rfp = np.linalg.norm((Mb @ y - x)[fp]) / np.linalg.norm(x[fp])
    print(f"{name} {extra}: s block {rs:.2e}  fp block {rfp:.2e}", flush=True)
    h.destroy()


def main():
    Nat.check(Nat.lib().pls_set_device(0))
    from oracle import synthetic as S
    for (d, N) in ((2, 16), (3, 5)):
        spec = S.SynthSpec(d, N)
        A, P = S.matrix(spec, 0), S.matrix(spec, 1)
        is_s, is_f, is_p = S.field_major_index_sets(spec)
        for extra in ({"pls.lu_path": "dense"}, {"pls.lu_path": "sparse"}, {"pls.lu_path": "sparse", "pls.lu_nd_leaf": "8"}):
            check(f"synthetic {d}-D N={N}", A, P, is_s, is_f, is_p, extra)
    from lib.fe_footing import assemble_footing
    for N in (8, 16):
        s = assemble_footing(N, "undrained")
        for extra in ({"pls.lu_path": "dense"}, {"pls.lu_path": "sparse"}, {"pls.lu_path": "band"}):
            check(f"footing N={N}", s.A, s.P, s.is_s, s.is_f, s.is_p, extra)


if __name__ == "__main__":
    main()
