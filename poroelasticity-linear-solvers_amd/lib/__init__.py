"""MI355X-native drop-in for the reference's solver layer (``lib/``).

Put ``poroelasticity-linear-solvers_amd/`` on ``sys.path`` and the reference's
drivers' ``from lib.Solver import Solver`` / ``from lib.Preconditioner import
Preconditioner`` resolve to these facades, which hand the assembled CSR blocks
to libpls.so (HIP kernels for gfx950) through include/pls.h.
"""
