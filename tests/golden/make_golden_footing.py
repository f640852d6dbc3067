"""Generate tests/golden/footing/*.npz: the oracle on footing systems
assembled by lib/fe_footing.py (footing.py's locally refined mesh, loads and
BCs; configs[2]).

The reference holds no fixtures; these pin the footing
assembler (mesh counts, matrix checksums) and the oracle on it against
regressions (tests/test_fe_footing.py; the device reproduces them in
tests/test_gpu_footing.py).  Regenerate with:
    python tests/golden/make_golden_footing.py
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poroelasticity-linear-solvers_amd")]

import bench  # noqa: E402
from lib.fe_footing import assemble_footing  # noqa: E402
from oracle.solver import OracleSolver  # noqa: E402

# footing.py:46-82 (solver atol 1e-4, maxiter 500, "pc type" undrained)
FOOTING_PARAMS = {"solver type": "gmres", "solver atol": 1e-4, "solver rtol": 1e-6, "solver maxiter": 500,
                  "pc type": "undrained", "inner rtol": 1e-6, "inner atol": 0, "inner maxiter": 1000,
                  "inner monitor": False, "solver monitor": False, "inner accel order": 0, "AAR order": 10,
                  "AAR p": 5, "AAR omega": 1, "AAR beta": 1}


def options(preset, pc="undrained"):
    """(params, db) of bench.py's preset on the footing driver's parameters:
    'exact' = petsc-options-exact (PREONLY + LU), 'inexact-ilu' = configs[2]'s
    set (petsc-options-inexact, BoomerAMG -> BJACOBI(ILU(0)) 64 blocks),
    'inexact' = petsc-options-inexact itself (hypre -> the classical AMG)."""
    ns = argparse.Namespace(solver="gmres", atol=1e-4, maxit=500, pc_type=pc, aar_order=10, blocks_inner=64,
                            inexact=preset == "inexact", preset=None if preset == "inexact" else preset, inner="ilu")
    params, db = bench.solver_options(ns)
    return dict(FOOTING_PARAMS, **params), db


CASES = {
    "footing_N8_undrained_exact": (8, "undrained", "exact"),
    "footing_N8_undrained_inexact_ilu": (8, "undrained", "inexact-ilu"),
    "footing_N8_3way_exact": (8, "diagonal 3-way", "exact"),
}


def checksums(s):
    out = []
    for M in (s.A, s.P, s.P_diff):
        out += [float(np.abs(M.data).sum()), float(M.data.sum())] if M is not None else [0.0, 0.0]
    return np.array(out + [float(np.abs(s.b).sum()), float(s.b.sum())])


def run_case(name):
    N, pc, preset = CASES[name]
    s = assemble_footing(N, pc)
    params, db = options(preset, pc)
    o = OracleSolver(s.A, s.P, s.P_diff, s.is_s, s.is_f, s.is_p, params, db, s.bcs_sub_pressure)
    x = o.solve(s.b)
    return s, params, db, o, x


def main():
    os.makedirs(os.path.join(HERE, "footing"), exist_ok=True)
    for name, (N, pc, preset) in CASES.items():
        s, params, db, o, x = run_case(name)
        meta = {"N": N, "pc": pc, "preset": preset, "params": params, "db": db}
        np.savez_compressed(os.path.join(HERE, "footing", name + ".npz"), meta=json.dumps(meta), its=o.its,
                            reason=o.reason, history=np.asarray(o.history), x=x, checksums=checksums(s),
                            dims=np.array(s.dims), nnz=s.A.nnz, bcs_sub_pressure=np.asarray(s.bcs_sub_pressure))
        print(f"{name:36s} n={s.A.shape[0]} nnz={s.A.nnz} its={o.its:3d} reason={o.reason}")


if __name__ == "__main__":
    main()
