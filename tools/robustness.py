"""The reference's own experiment (paper-scripts/robustness_2d.sh) on the device.

robustness_2d.sh runs, under ``mpirun -np 8``:
  * swelling.py -N {10,20,40,80,160} --pc-type "diagonal" / "diagonal 3-way"
  * footing.py  -N {10,20,40,80}     --pc-type "undrained" / "undrained 3-way"
each with petsc-options-exact and petsc-options-inexact, and records the
outer iteration count (lib/AbstractPhysics.py:77-78: "... {its} iterations").

Here every case runs the reference's call sequence through the facade
(lib/Preconditioner.py -> get_pc, lib/Solver.py -> create_solver, set_up,
solve; lib/Poromechanics.py:58-98) on the system lib/fe_swelling.py /
lib/fe_footing.py assemble for the first time step (dt = tf = 0.1: one step),
with the drivers' own parameter dictionaries (swelling.py:44-85,
footing.py:44-92) and the option files (options/exact, options/inexact).

np = 8 semantics (--np 8, the default): MUMPS's LU does not depend on the
rank count; BoomerAMG does -- HMIS coarsens inside each of the 8 processes and
relaxes with hybrid Gauss-Seidel, Gauss-Seidel inside a process and Jacobi
across them (one OpenMP thread per rank: 8 chunks).  That is
pls.hypre_ranks 8 + pls.hypre_relax_chunks 8: each block's rows cut into 8
contiguous ranks.  (Under mpirun, dolfin numbers the dofs after a ParMETIS
partition of the mesh; the ranks' rows here are contiguous ranges of the
assembler's RCM order instead -- the partition itself is not reproducible
without dolfin.)

usage: python tools/robustness.py --problem swelling --N 10 20 --pc "diagonal" --set exact
           [--np 8] [--out gpurun_out/robustness.jsonl] [--oracle]
Each case prints one JSON line and appends it to --out.  --oracle also
solves the case with the CPU oracle (small N only) and records its count.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "poroelasticity-linear-solvers_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

# the drivers' solver parameters (swelling.py:62-80, footing.py:66-84); the
# option files override the inner solver types (setFromOptions)
_COMMON = {"solver type": "gmres", "solver monitor": False, "inner ksp type": "gmres", "inner pc type": "hypre",
           "inner atol": 0, "inner rtol": 1e-6, "inner maxiter": 1000, "inner monitor": False,
           "inner accel order": 0, "AAR order": 10, "AAR p": 5, "AAR omega": 1, "AAR beta": 1}
DRIVER = {
    "swelling": dict(_COMMON, **{"solver atol": 1e-8, "solver rtol": 1e-6, "solver maxiter": 500}),
    "footing": dict(_COMMON, **{"solver atol": 1e-4, "solver rtol": 1e-6, "solver maxiter": 500}),
}
INNER = ("s_", "f_", "p_", "diff_", "fp_", "fp_fieldsplit_0_", "fp_fieldsplit_1_")


def np_options(nranks: int) -> dict:
    """BoomerAMG as mpirun -np nranks runs it (one thread per rank)."""
    if nranks <= 1:
        return {"pls.hypre_relax_chunks": "1"}
    return {"pls.hypre_ranks": str(nranks), "pls.hypre_relax_chunks": str(nranks)}


def load_set(name: str) -> dict:
    from lib import options as popts
    from lib.Parser import load_options_file
    popts.DB.clear()
    load_options_file(os.path.join(ROOT, "options", name))
    return dict(popts.DB)


def assemble(problem: str, N: int, pc: str):
    if problem == "swelling":
        from lib.fe_swelling import assemble_swelling
        return assemble_swelling(2, N, pc)
    from lib.fe_footing import assemble_footing
    return assemble_footing(N, pc)


def run_case(problem: str, N: int, pc: str, optset: str, nranks: int, extra: dict | None = None,
             oracle: bool = False, history: bool = False) -> dict:
    from lib import options as popts
    from lib.IndexSet import IndexSet
    from lib.Preconditioner import Preconditioner
    from lib.Solver import Solver
    t0 = time.time()
    s = assemble(problem, N, pc)
    t_asm = time.time() - t0
    params = dict(DRIVER[problem], **{"pc type": pc})
    db = load_set(optset)
    db.update(np_options(nranks))
    db.update(extra or {})
    popts.DB.clear()
    popts.DB.update(db)
    three = "3-way" in pc
    index_map = IndexSet((s.is_s, s.is_f, s.is_p), two_way=not three)
    t1 = time.time()
    prec = Preconditioner(index_map, s.A, s.P, s.P_diff if three else None, params, s.bcs_sub_pressure)
    pcobj = prec.get_pc()
    b = s.b.copy()
    solver = Solver(s.A, b, pcobj, params, index_map)
    solver.create_solver(s.A, b, pcobj)
    solver.set_up()
    t_setup = time.time() - t1
    x = np.zeros_like(b)
    t2 = time.time()
    # heartbeat while the library solves (ctypes releases the GIL): long cases
    # must keep writing or the GPU harness takes them for hung
    import threading
    done = threading.Event()

    def beat():
        while not done.wait(30):
            print(f"[robustness] {problem} N={N} '{pc}' {optset}: solving, {time.time() - t2:.0f} s", flush=True)
    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        solver.solve(b, x)
    finally:
        done.set()
        th.join()
    t_solve = time.time() - t2
    h = pcobj.handle
    inner = {}
    for pre in INNER:
        try:
            st = h.ksp_stats(pre)
        except RuntimeError:
            continue
        if st[0]:
            inner[pre] = {"solves": st[0], "its": st[1], "max": st[2], "negative_reason": st[3],
                          "last_negative": st[4]}
    hist = solver.history
    out = {"problem": problem, "N": N, "pc_type": pc, "options": optset, "np": nranks, "dofs": int(s.A.shape[0]),
           "nnz": int(s.A.nnz), "its": int(solver.getIterationNumber()), "reason": int(solver.getConvergedReason()),
           "rnorm0": float(hist[0]) if hist.size else None, "rnorm": float(hist[-1]) if hist.size else None,
           "assembly_s": round(t_asm, 2), "setup_s": round(t_setup, 2), "solve_s": round(t_solve, 3),
           "inner": inner, "extra": extra or {}}
    if history:
        out["history"] = [float(v) for v in hist]
    h.destroy()
    if oracle:
        from oracle.solver import OracleSolver
        t3 = time.time()
        o = OracleSolver(s.A, s.P, s.P_diff if three else None, s.is_s, s.is_f, s.is_p, params, db,
                         s.bcs_sub_pressure)
        o.solve(s.b)
        ho = np.asarray(o.history)
        m = min(ho.size, hist.size)
        out["oracle"] = {"its": int(o.its), "reason": int(o.reason), "s": round(time.time() - t3, 1),
                         "history_rel_diff": float(np.max(np.abs(hist[:m] - ho[:m]) / ho[:m])) if m else None}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problem", choices=["swelling", "footing"], required=True)
    ap.add_argument("--N", type=int, nargs="+", required=True)
    ap.add_argument("--pc", nargs="+", required=True)
    ap.add_argument("--set", nargs="+", default=["exact", "inexact"])
    ap.add_argument("--np", type=int, default=8)
    ap.add_argument("--opt", action="append", default=[], help="extra library option key=value")
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--monitor", action="store_true", help="print every outer iteration's residual (-global_ksp_monitor)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "robustness.jsonl"))
    a = ap.parse_args()
    import lib._native as Nat
    Nat.check(Nat.lib().pls_set_device(0))
    extra = dict(kv.split("=", 1) for kv in a.opt)
    if a.monitor:
        extra["global_ksp_monitor"] = None
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    for optset in a.set:
        for N in a.N:
            for pc in a.pc:
                r = run_case(a.problem, N, pc, optset, a.np, extra, a.oracle)
                line = json.dumps(r)
                print(line, flush=True)
                with open(a.out, "a") as f:
                    f.write(line + "\n")


if __name__ == "__main__":
    main()
