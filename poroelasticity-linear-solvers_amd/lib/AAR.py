"""Anderson-accelerated Richardson facade (reference lib/AAR.py).

``AAR(order, p, omega, beta, matA, x0=None, pc=None, atol, rtol, maxiter,
monitor_convergence)`` with ``solve(b, sol) -> it`` and ``getIterationNumber``.
The iteration (46-128) runs in libpls.so on the PC's handle (the operator is
the handle's A, which must be ``matA``); the Anderson least squares replaces the
rank-0 numpy QR of full gathered vectors (85-108) with a device Householder
TSQR whose per-rank (order+1)^2 R factors are all-gathered.  As in the reference, ``pc=None`` is an error
(the reference dereferences an undefined ``self.solver`` at 33-38).
"""
from ._native import vec_array


class AAR:
    def __init__(self, order, p, omega, beta, matA, x0=None, pc=None, atol=1e-12, rtol=1e-8, maxiter=1000,
                 monitor_convergence=False):
        self.order, self.p, self.omega, self.beta = order, p, omega, beta
        self.matA = matA
        self.x0 = x0
        self.atol, self.rtol, self.maxiter = atol, rtol, maxiter
        self.monitor_convergence = monitor_convergence
        if not pc:
            raise AttributeError("'AAR' object has no attribute 'solver' (AAR needs a preconditioner)")
        self.pc = pc
        self.it = 0
        h = pc.handle
        for k, v in (("pls.solver_type", "aar"), ("pls.aar_order", order), ("pls.aar_p", p),
                     ("pls.aar_omega", omega), ("pls.aar_beta", beta), ("pls.solver_atol", atol),
                     ("pls.solver_rtol", rtol), ("pls.solver_maxiter", maxiter),
                     ("pls.solver_monitor", 1 if monitor_convergence else 0)):
            h.set_option(k, v)
        h.create_solver()
        self.history = None

    def set_up(self):
        pass

    def solve(self, b, sol):
        xs, r = self.pc.handle.solve(vec_array(b))
        sa = vec_array(sol)
        sa[...] = xs
        self.it = r.its
        self.history = self.pc.handle.history()
        return self.it

    def getIterationNumber(self):
        return self.it
