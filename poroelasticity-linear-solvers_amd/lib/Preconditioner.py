"""Block preconditioner facade (reference lib/Preconditioner.py).

``Preconditioner(index_map, A, P, P_diff, parameters, bcs_sub_pressure)``
validates the pc type exactly like the reference (263-280, ``sys.exit`` with
the same message) and ``get_pc()`` builds the PC (282-291).  The work --
sub-block extraction, inner KSP/PC setup (s_ f_ p_ diff_ fp_ prefixes, options
win), and every ``apply`` (2-way 219-246, 3-way 150-218, inner Anderson
248-249) -- runs in libpls.so on the GPU.  Inside a multi-rank job
(torch.distributed initialised with world size G, the reference's
``mpirun -np G``) the matrices are taken as this rank's rows and the handle is
sharded over ``lib.dist.default_communicator()`` (pls_create_dist).
"""
from time import perf_counter as time

from . import options as _opts
from ._native import csr_of, vec_array
from .dist import default_communicator
from .handle import Handle, params_to_options
from .Printing import parprint

PC_TYPES = ("undrained", "undrained 3-way", "diagonal", "diagonal 3-way", "diagonal 3-way-II", "lu")


def _fingerprint(M):
    """Cheap value/pattern fingerprint of a matrix-like (scipy / petsc4py / dolfin)."""
    import numpy as np
    if M is None:
        return None
    ai, aj, av, nr, nc = csr_of(M)
    return (nr, nc, av.size, float(np.sum(av)), float(np.dot(av, av)), int(np.sum(aj, dtype=np.int64)))


class PreconditionerCC(object):
    """The python-PC context: ``setUp(pc)`` / ``apply(pc, x, y)`` / ``print_timings``."""

    def __init__(self, handle: Handle, flag_3_way: bool, mats=(None, None, None)):
        self.handle = handle
        self.mats = mats
        self._prints = None
        self.flag_3_way = flag_3_way

    def setUp(self, pc=None):
        t0 = time()
        self.handle.setup()
        parprint("---- [Preconditioner] Set up in {}s".format(time() - t0))

    def refresh(self):
        """Re-set-up after A / P / P_diff changed in place (the reference's
        bc.apply + PCSetUp every time step, lib/Poromechanics.py:70-86)."""
        prints = tuple(_fingerprint(M) for M in self.mats)
        if self._prints is None:
            self._prints = prints
            return False
        changed = [m if p != q else None for m, p, q in zip(self.mats, prints, self._prints)]
        self._prints = prints
        if any(c is not None for c in changed):
            self.handle.update_matrices(*changed)
            return True
        return False

    def apply(self, pc, x, y):
        """y = M^{-1} x (host vectors in the caller's ordering)."""
        yy = self.handle.pc_apply(vec_array(x))
        ya = vec_array(y)
        ya[...] = yy
        return y

    def print_timings(self):
        t = self.handle.timings()
        parprint("\n===== Timing preconditioner: {:.3f}s".format(t["pc_total"]))
        if self.flag_3_way:
            parprint("\tSolid solver: {:.3f}s\n\tFluid solver: {:.3f}s\n\tPressure solver: {:.3f}s".format(
                t["pc_solid"], t["pc_fluid"], t["pc_press"]))
        else:
            parprint("\tSolid solver: {:.3f}s\n\tFluid-pressure solver: {:.3f}s".format(t["pc_solid"], t["pc_fluid"]))
        parprint("\n\tAllocation time: {:.3f}".format(t["pc_alloc"]))


class PC:
    """What ``get_pc()`` returns: ``apply(x, y)``, ``setUp()``, ``getPythonContext()``."""

    def __init__(self, ctx: PreconditionerCC):
        self._ctx = ctx
        self.handle = ctx.handle

    def setUp(self):
        self._ctx.setUp(self)

    def apply(self, x, y):
        return self._ctx.apply(self, x, y)

    def getPythonContext(self):
        return self._ctx

    def getType(self):
        return "python"


class Preconditioner:
    def __init__(self, index_map, A, P, P_diff, parameters, bcs_sub_pressure):
        self.index_map = index_map
        self.A = A
        self.P = P
        self.P_diff = P_diff
        self.parameters = parameters
        self.pc_type = parameters["pc type"]
        self.inner_ksp_type = parameters["inner ksp type"]
        self.inner_pc_type = parameters["inner pc type"]
        self.inner_rtol = parameters["inner rtol"]
        self.inner_atol = parameters["inner atol"]
        self.inner_maxiter = parameters["inner maxiter"]
        self.inner_accel_order = parameters["inner accel order"]
        self.inner_monitor = parameters["inner monitor"]
        self.bcs_sub_pressure = bcs_sub_pressure
        if self.pc_type not in PC_TYPES:
            import sys
            sys.exit("pc type must be one of lu, undrained, diagonal, diagonal 3-way, diagonal 3-way-II.")

    def get_pc(self):
        flag_3_way = self.pc_type in ("diagonal 3-way", "undrained 3-way")
        is_s, is_f, is_p = self.index_map.global_index_sets()
        opts = dict(_opts.DB)
        opts.update(params_to_options(self.parameters))
        comm = default_communicator()
        if comm is not None:
            # one rank of G (mpirun -np G in the reference): the matrices are this
            # rank's rows, the index sets the dofs it owns (pls_create_dist)
            handle = Handle.from_csr_dist(self.A, self.P, self.P_diff if flag_3_way else None, is_s, is_f, is_p,
                                          self.bcs_sub_pressure, opts, comm)
        else:
            handle = Handle.from_csr(self.A, self.P, self.P_diff if flag_3_way else None, is_s, is_f, is_p,
                                     self.bcs_sub_pressure, opts)
        ctx = PreconditionerCC(handle, flag_3_way, (self.A, self.P, self.P_diff if flag_3_way else None))
        self.pc = PC(ctx)
        self.pc.setUp()
        return self.pc

    def print_timings(self):
        ctx = self.pc.getPythonContext()
        ctx.print_timings()
