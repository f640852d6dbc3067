"""Golden data for tests/test_gpu_harness.py: the CPU oracle on the reference
harness's cases at N = 10 (paper-scripts/robustness_2d.sh: swelling.py and
footing.py, 2-way and 3-way pc types, petsc-options-exact and -inexact, with
mpirun -np 8's BoomerAMG semantics -- tools/robustness.py).

Per case: the oracle's iteration count, reason and residual history, and its
iteration counts when every inner PC output is perturbed by 1e-15 relative
(6 seeds): where those counts spread, the case's count is set by rounding
(non-normal saddle-point systems, nonlinear inner CG solves inside GMRES) and
the device is held to that range, not to one value.  On the exact option set
the oracle is also run with its sparse LU (scipy splu, COLAMD) under two other
column orderings (NATURAL, MMD(A^T + A)): two backward-stable exact solves, as
MUMPS and the device LU are (tests/test_gpu_fe.py _lu_swap_floor).  Stored:

* ``lu_swap_floor``: the largest relative history deviation of those LU-swap
  runs where the count does not move (the exact sets' history bound is 10x
  that, at least 1e-10);
* ``first_dev``: per perturbation run (eps seeds, then LU swaps), the first
  iteration whose residual deviates from the unperturbed history by more than
  1e-10 relative (its length when none does); the device history is held to
  1e-10 up to the smallest of them on the cases whose count moves -- on the
  exact set to 10x ``lu_swap_prefix_floor``, the LU-swap runs' largest
  relative deviation over that prefix, if larger (the device LU is a third
  backward-stable LU: it moves the history as much as the swaps do).

usage: python tests/golden/harness/make_golden_harness.py  (writes n10.json)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
for p in (ROOT, os.path.join(ROOT, "poroelasticity-linear-solvers_amd"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)

import robustness as R  # noqa: E402
from oracle.solver import OracleSolver  # noqa: E402

CASES = [(prob, pc, optset) for optset in ("exact", "inexact")
         for prob, pcs in (("swelling", ("diagonal", "diagonal 3-way")), ("footing", ("undrained", "undrained 3-way")))
         for pc in pcs]


TOL = 1e-10


def first_dev(h, ho, tol=TOL):
    """First index where h deviates from ho by more than tol relative (the
    common length when it never does; a differing length counts from there)."""
    h, ho = np.asarray(h), np.asarray(ho)
    m = min(h.size, ho.size)
    bad = np.flatnonzero(np.abs(h[:m] - ho[:m]) > tol * np.abs(ho[:m]))
    return int(bad[0]) if bad.size else m


def run(prob, pc, optset, N=10, seed=None, eps=1e-15, lu_spec=None):
    if lu_spec is not None:
        import scipy.sparse as sp
        import scipy.sparse.linalg as spla
        from oracle import petsc as OP
        orig = OP.PCLU.__init__

        def init(self, M):
            self.f = spla.splu(sp.csc_matrix(M), permc_spec=lu_spec)
        OP.PCLU.__init__ = init
        try:
            return run(prob, pc, optset, N, seed, eps)
        finally:
            OP.PCLU.__init__ = orig
    s = R.assemble(prob, N, pc)
    params = dict(R.DRIVER[prob], **{"pc type": pc})
    db = R.load_set(optset)
    db.update(R.np_options(8))
    three = "3-way" in pc
    o = OracleSolver(s.A, s.P, s.P_diff if three else None, s.is_s, s.is_f, s.is_p, params, db, s.bcs_sub_pressure)
    if seed is not None:
        rng = np.random.default_rng(seed)
        for name in ("ksp_s", "ksp_fp", "ksp_f", "ksp_p", "ksp_p_diff"):
            ksp = getattr(o.block_pc, name, None)
            if ksp is not None:
                f = ksp.pc.apply
                ksp.pc.apply = (lambda f: lambda x: (lambda y: y * (1 + eps * rng.standard_normal(y.size)))(f(x)))(f)
    o.solve(s.b)
    return o


def main():
    out = {}
    for prob, pc, optset in CASES:
        o = run(prob, pc, optset)
        runs = [run(prob, pc, optset, seed=k) for k in range(6)]
        swaps = [run(prob, pc, optset, lu_spec=spec) for spec in ("NATURAL", "MMD_AT_PLUS_A")] \
            if optset == "exact" else []
        ho = np.asarray(o.history)
        floor = 0.0
        for q in swaps:
            if q.its == o.its:
                floor = max(floor, float(np.max(np.abs(np.asarray(q.history) - ho) / ho)))
        k = min(first_dev(q.history, ho) for q in runs + swaps)
        pfloor = 0.0
        for q in swaps:
            hq = np.asarray(q.history)
            m = min(k, hq.size, ho.size)
            if m:
                pfloor = max(pfloor, float(np.max(np.abs(hq[:m] - ho[:m]) / ho[:m])))
        key = f"{prob}|{pc}|{optset}"
        out[key] = {"its": int(o.its), "reason": int(o.reason), "history": [float(v) for v in o.history],
                    "perturbed_its": [int(q.its) for q in runs],
                    "lu_swap_its": [int(q.its) for q in swaps],
                    "lu_swap_floor": floor,
                    "lu_swap_prefix_floor": pfloor,
                    "first_dev": [first_dev(q.history, ho) for q in runs + swaps]}
        print(key, o.its, out[key]["perturbed_its"], out[key]["lu_swap_its"], floor, out[key]["first_dev"],
              flush=True)
    with open(os.path.join(HERE, "n10.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
