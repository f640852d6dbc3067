"""Outer solver facade (reference lib/Solver.py).

``Solver(A, b, PC, parameters, index_map)``; ``create_solver`` configures the
outer KSP (prefix ``global_``, type, ``setTolerances(rtol, atol, 1e20,
maxiter)``, GMRES restart = maxiter, options win: 91-102) or AAR (84-90);
``solve(b, x)`` runs the whole Krylov loop in libpls.so; ``set_up`` keeps the
reference's no-op convergence-argument preparation (105-143).  The reference's
custom ``converged`` test (8-51) is never installed there, so it is not here.
"""
from time import perf_counter as time

import numpy as np

from . import options as _opts
from ._native import vec_array
from .handle import params_to_options
from .Printing import parprint


class Solver:
    def __init__(self, A, b, PC, parameters, index_map):
        self.A = A
        self.b = b
        self.PC = PC
        self.solver = None
        self.parameters = parameters
        self.index_map = index_map
        self.t_total = 0
        self.its = 0
        self.reason = 0
        self.history = np.zeros(0)

    def create_solver(self, A, b, PC):
        t0_create = time()
        h = self.PC.handle
        opts = {k: v for k, v in _opts.DB.items() if k.startswith("global_")}
        opts.update({k: v for k, v in params_to_options(self.parameters).items()
                     if k.startswith("pls.solver") or k.startswith("pls.aar")})
        for k, v in opts.items():
            h.set_option(k, v)
        h.create_solver()
        self.solver = h
        parprint("---- [Solver] Solver created in {}s".format(time() - t0_create))

    def set_up(self):
        """KSPSetUp (lib/Solver.py:105-143): the PC is set up again when A / P /
        P_diff changed since the last set_up (PETSc's operator-state check)."""
        t0_setup = time()
        ctx = getattr(self.PC, "getPythonContext", lambda: None)()
        if ctx is not None and hasattr(ctx, "refresh"):
            ctx.refresh()
        parprint("---- [Solver] Solver set up in {}s".format(time() - t0_setup))

    def getIterationNumber(self):
        return self.its

    def getConvergedReason(self):
        return self.reason

    def solve(self, b, x):
        t0 = time()
        xs, r = self.solver.solve(vec_array(b))
        xa = vec_array(x)
        xa[...] = xs
        self.its, self.reason = r.its, r.reason
        self.history = self.solver.history()
        self.t_total += time() - t0

    def print_timings(self):
        parprint("\n===== Timing Solver: {:.3f}s".format(self.t_total))
