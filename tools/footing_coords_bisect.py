"""Why footing N=12's iteration count moved from 53 to 39 during round 3 (CPU only).

Commit a5b2e1c changed lib/fe_footing.py's grid coordinates from
i * (length / N) to (i / N) * length (UnitSquareMesh, then `*= length`,
reference lib/MeshCreation.py:17-19).  This script assembles the footing
system both ways, prints the matrix checksums, the number of triangles whose
vertex sets differ after the two Plaza refinements, and the oracle's outer
iteration count with footing.py's own option set (petsc-options-inexact).

    python tools/footing_coords_bisect.py [N]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poroelasticity-linear-solvers_amd"), os.path.join(ROOT, "tests", "golden")]

from lib import fe_footing as FF  # noqa: E402
from lib import fe_swelling as F  # noqa: E402


def mesh(N, old, length=FF.LENGTH):
    ic, cells = F.unit_mesh(2, N)
    coords = ic.astype(np.float64) * (length / N) if old else (ic.astype(np.float64) / N) * length
    for _ in range(2):
        x, y = coords[cells, 0], coords[cells, 1]
        mark = (y.min(1) > 2 * length / 3) & (x.min(1) > length / 8) & (x.max(1) < 7 / 8 * length)
        coords, cells = FF.plaza_refine(coords, cells, mark)
    return coords, cells


def cell_set(coords, cells):
    key = np.round(coords * 3000).astype(np.int64)
    return {frozenset(map(tuple, key[c])) for c in cells}


def main():
    import make_golden_footing as G
    from oracle.solver import OracleSolver
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    (co, ko), (cn, kn) = mesh(N, True), mesh(N, False)
    print(f"N={N}: vertices {len(co)} / {len(cn)}, triangles {len(ko)} / {len(kn)}, "
          f"triangles not in both: {len(cell_set(co, ko) ^ cell_set(cn, kn))}")
    orig = FF.footing_mesh
    for name, old in (("i*(L/N)", True), ("(i/N)*L", False)):
        FF.footing_mesh = lambda n, length=FF.LENGTH, refinements=0, _old=old: mesh(n, _old, length)
        try:
            s = FF.assemble_footing(N, "undrained")
        finally:
            FF.footing_mesh = orig
        params, db = G.options("inexact")
        o = OracleSolver(s.A, s.P, s.P_diff, s.is_s, s.is_f, s.is_p, params, db, s.bcs_sub_pressure)
        o.solve(s.b)
        cs = G.checksums(s)
        print(f"  {name}: n={s.A.shape[0]} nnz={s.A.nnz} sum|A|={cs[0]:.6e} sum|P|={cs[2]:.6e} "
              f"oracle its={o.its} reason={o.reason}")


if __name__ == "__main__":
    main()
