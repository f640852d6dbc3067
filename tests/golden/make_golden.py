"""Generate the golden fixtures tests/golden/*.npz from the CPU oracle.

The reference holds no golden vectors, so these fixtures are
produced by the oracle on seeded synthetic systems and pin both the oracle
(tests/test_golden.py, CPU) and libpls.so (GPU) against regressions.  Each file
stores the configuration, iteration count, convergence reason, residual
history and the solution.  Regenerate with:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import synthetic as S  # noqa: E402
from oracle.solver import OracleSolver  # noqa: E402

BASE = {"solver type": "gmres", "solver atol": 1e-8, "solver rtol": 1e-6, "solver maxiter": 300,
        "pc type": "diagonal", "inner ksp type": "preonly", "inner pc type": "ilu", "inner accel order": 0,
        "AAR order": 10, "AAR p": 5, "AAR omega": 1, "AAR beta": 1}
PRE = ("s_", "f_", "p_", "diff_", "fp_")


def db_of(pc, side="right", extra=None):
    db = {"global_ksp_type": "gmres"}
    if side:
        db["global_ksp_pc_side"] = side
    for p in PRE:
        db[p + "ksp_type"] = "preonly"
        db[p + "pc_type"] = pc
    db.update(extra or {})
    return db


CASES = {
    "gmres_right_2way_ilu_2d": ((2, 8), {}, db_of("ilu")),
    "gmres_left_2way_ilu_2d": ((2, 8), {}, db_of("ilu", side=None)),
    "gmres_right_3way_ilu_2d": ((2, 8), {"pc type": "diagonal 3-way"}, db_of("ilu")),
    "gmres_right_2way_lu_2d": ((2, 6), {"inner pc type": "lu"}, db_of("lu")),
    "gmres_right_3way_lu_2d": ((2, 6), {"pc type": "diagonal 3-way", "inner pc type": "lu"}, db_of("lu")),
    "gmres_right_2way_bjacobi_3d": ((3, 2), {}, db_of("bjacobi", extra={p + "pc_bjacobi_blocks": "4" for p in PRE})),
    "gmres_right_2way_jacobi_3d": ((3, 2), {}, db_of("jacobi")),
    "gmres_inner_cg_2d": ((2, 8), {}, db_of("ilu", extra={"s_ksp_type": "cg", "s_ksp_rtol": "1e-1",
                                                          "s_ksp_norm_type": "unpreconditioned",
                                                          "fp_ksp_type": "gmres", "fp_ksp_rtol": "1e-2"})),
    "aar_2way_ilu_2d": ((2, 8), {"solver type": "aar", "solver maxiter": 200}, db_of("ilu")),
}


def run_case(name):
    (dim, N), upd, db = CASES[name]
    spec = S.SynthSpec(dim, N)
    params = dict(BASE)
    params.update(upd)
    A, P, Pd = S.matrix(spec, 0), S.matrix(spec, 1), S.matrix(spec, 2)
    is_s, is_f, is_p = S.field_major_index_sets(spec)
    o = OracleSolver(A, P, Pd, is_s, is_f, is_p, params, db, S.bcs_sub_pressure(spec))
    x = o.solve(S.rhs(spec))
    return spec, params, db, o, x


def main():
    for name in CASES:
        spec, params, db, o, x = run_case(name)
        meta = {"dim": spec.dim, "N": spec.N, "seed": spec.seed, "delta": spec.delta, "params": params, "db": db}
        np.savez_compressed(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta), its=o.its, reason=o.reason,
                            history=np.asarray(o.history), x=x)
        print(f"{name:34s} its={o.its:3d} reason={o.reason}")


if __name__ == "__main__":
    main()
