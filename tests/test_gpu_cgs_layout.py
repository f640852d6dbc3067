"""The classical Gram-Schmidt kernels of the GMRES cycle (lib/Solver.py's
PETSc GMRES, CGS orthogonalisation) in their two device forms: column-streamed
(`k_mdot_cols` / `k_maxpy_norm_cols`, the default while a block's chunk fits
the registers) and row-interleaved (`k_mdot` / `k_maxpy_norm`, forced with
PLS_MDOT_ROWS).  Per (column, thread) both sum in the same order, so a whole
solve -- residual history and solution -- is bitwise the same."""
import os

import numpy as np
import pytest

from lib.handle import Handle, params_to_options
from oracle import synthetic as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dim,N", [(3, 6), (2, 40)])
def test_cgs_column_streams_bitwise_equal_row_interleaved(dim, N):
    spec = S.SynthSpec(dim, N)
    opts = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "s_ksp_type": "preonly",
            "s_pc_type": "bjacobi", "fp_ksp_type": "preonly", "fp_pc_type": "bjacobi"}
    opts.update(params_to_options({"solver type": "gmres", "solver atol": 1e-12, "solver rtol": 1e-10,
                                   "solver maxiter": 200, "pc type": "diagonal", "inner ksp type": "preonly",
                                   "inner pc type": "bjacobi"}))
    b = S.rhs(spec)
    out = []
    for rows in (False, True):
        if rows:
            os.environ["PLS_MDOT_ROWS"] = "1"
        try:
            h = Handle.synthetic(spec.dim, spec.N, spec.seed, spec.delta, opts)
            x, r = h.solve(b)
            out.append((x, r.its, h.history()))
            h.destroy()
        finally:
            os.environ.pop("PLS_MDOT_ROWS", None)
    (x0, i0, h0), (x1, i1, h1) = out
    assert i0 == i1 and i0 > 30  # (past one restart cycle: columns up to 30)
    assert np.array_equal(h0, h1) and np.array_equal(x0, x1)
