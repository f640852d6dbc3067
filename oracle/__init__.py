"""CPU oracle for the block-preconditioned Krylov hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import anything from this package, and
only as the checker (or the timed CPU baseline).  The product path
(``poroelasticity-linear-solvers_amd/``, ``libpls.so``) never imports, links or
calls it, and fails loudly when its HIP library is missing.

What it restates (each function cites the reference file:line it follows):

* ``petsc``      PETSc KSP/PC semantics exactly as the reference configures
                 them: GMRES (CGS, Givens, BuildSoln, restart) and CG as run by
                 ``KSPSolve`` (reference ``lib/Solver.py:91-102,151``),
                 ``KSPConvergedDefault``, PREONLY, and the inner PCs
                 NONE/JACOBI/ILU(0)/BJACOBI/LU (``lib/Preconditioner.py:94-118``).
* ``blockpc``    ``PreconditionerCC`` 2-way / 3-way apply
                 (reference ``lib/Preconditioner.py:141-250``).
* ``aar``        ``AAR.solve`` and ``AndersonAcceleration.get_next_vector``
                 (reference ``lib/AAR.py:46-137``, ``lib/AndersonAcceleration.py:19-78``).
* ``options``    the options-file loader (reference ``lib/Parser.py:61-73``) and
                 the prefix/precedence rules of ``setFromOptions``.
* ``index_sets`` the 2-way fp re-indexing (reference ``lib/IndexSet.py:10-26,46-54``).
* ``synthetic``  the seeded synthetic 3-field system of SURVEY.md 8(d).
* ``csrc/oracle.c`` C kernels for the parts numpy cannot do at speed
                 (synthetic generator, MatMult, ILU(0) factor and MatSolve).

PARITY STATUS -- "parity unpinned" against the reference itself.  The
reference is pure Python over petsc4py/dolfin/MUMPS/hypre, none of which exist
in this image (ordinary ModuleNotFoundError, not a permission
denial), it holds no tests, golden vectors or fixtures, and PETSc is a
third-party dependency with no pinned version (the code implies PETSc >= 3.9 by
its ``pc_factor_mat_solver_type`` spelling).  The PETSc algorithms above are
restated from PETSc's published source semantics (gmres.c, cg.c, aij.c,
bjacobi.c, iterativ.c) and each is pinned by independent known-answer tests
in ``tests/test_oracle.py``: scipy ``A @ x`` and ``splu`` for MatMult/LU,
hand-computed 3x3 GMRES/ILU cases, exact-solution convergence, and a dense
numpy GMRES/least-squares restatement.  The golden fixtures under
``tests/golden/`` are generated from this oracle (``tests/golden/make_golden.py``).
"""
