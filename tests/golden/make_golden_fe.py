"""Generate tests/golden/fe/*.npz: the oracle on systems assembled by
lib/fe_swelling.py (true swelling operators).

The reference holds no fixtures; these pin the assembler
(matrix checksums) and the oracle on it against regressions
(tests/test_fe_swelling.py).  Regenerate with:
    python tests/golden/make_golden_fe.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poroelasticity-linear-solvers_amd")]

from lib.fe_swelling import assemble_swelling  # noqa: E402
from oracle.solver import OracleSolver  # noqa: E402

BASE = {"solver type": "gmres", "solver atol": 1e-8, "solver rtol": 1e-6, "solver maxiter": 300,
        "pc type": "diagonal", "inner ksp type": "preonly", "inner pc type": "lu", "inner rtol": 1e-6,
        "inner atol": 0, "inner maxiter": 1000, "inner monitor": False, "solver monitor": False,
        "inner accel order": 0, "AAR order": 10, "AAR p": 5, "AAR omega": 1, "AAR beta": 1}


def db_of(pc):
    db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right"}
    for p in ("s_", "f_", "p_", "diff_", "fp_"):
        db[p + "ksp_type"] = "preonly"
        db[p + "pc_type"] = pc
    return db


CASES = {
    "fe_swelling2d_N6_diagonal_lu": (2, 6, "diagonal", "lu"),
    "fe_swelling2d_N6_3way_ilu": (2, 6, "diagonal 3-way", "ilu"),
    "fe_swelling3d_N2_diagonal_ilu": (3, 2, "diagonal", "ilu"),
}


def checksums(s):
    out = []
    for M in (s.A, s.P, s.P_diff):
        out += [float(np.abs(M.data).sum()), float(M.data.sum())] if M is not None else [0.0, 0.0]
    return np.array(out + [float(np.abs(s.b).sum())])


def run_case(name):
    dim, N, pc, inner = CASES[name]
    s = assemble_swelling(dim, N, pc)
    params = dict(BASE, **{"pc type": pc})
    db = db_of(inner)
    o = OracleSolver(s.A, s.P, s.P_diff, s.is_s, s.is_f, s.is_p, params, db, s.bcs_sub_pressure)
    x = o.solve(s.b)
    return s, params, db, o, x


def main():
    os.makedirs(os.path.join(HERE, "fe"), exist_ok=True)
    for name, (dim, N, pc, inner) in CASES.items():
        s, params, db, o, x = run_case(name)
        meta = {"dim": dim, "N": N, "pc": pc, "params": params, "db": db}
        np.savez_compressed(os.path.join(HERE, "fe", name + ".npz"), meta=json.dumps(meta), its=o.its,
                            reason=o.reason, history=np.asarray(o.history), x=x, checksums=checksums(s))
        print(f"{name:34s} its={o.its:3d} reason={o.reason}")


if __name__ == "__main__":
    main()
