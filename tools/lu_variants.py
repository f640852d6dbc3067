"""Diagnostics: unrefined ||K y - x|| / ||x|| of the sparse LU on the blocks of a
small assembled system for a list of option variants (ordering, leaf size,
static pivoting), to locate shape-dependent accuracy problems on the device.

usage: python tools/lu_variants.py [footing8|swelling2d8] [key=value,key=value ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poroelasticity-linear-solvers_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import lib._native as Nat  # noqa: E402
from test_gpu_sparse_lu import _block_residuals, _handle  # noqa: E402


def main():
    Nat.check(Nat.lib().pls_set_device(0))
    system = sys.argv[1] if len(sys.argv) > 1 else "footing8"
    if system.startswith("footing"):
        from lib.fe_footing import assemble_footing
        s = assemble_footing(int(system[7:]), "undrained")
    else:
        from lib.fe_swelling import assemble_swelling
        s = assemble_swelling(2, int(system[11:]), "diagonal")
    x = np.random.default_rng(5).standard_normal(s.A.shape[0])
    variants = sys.argv[2:] or ["pls.lu_nd_leaf=64", "pls.lu_nd_leaf=8"]
    for v in variants:
        extra = dict(kv.split("=", 1) for kv in v.split(",")) if v else {}
        extra.setdefault("pls.lu_refine", "0")
        h = _handle(s, extra)
        y = h.pc_apply(x)
        h.destroy()
        rs, rfp = _block_residuals(s, y, x)
        print(f"{system} {extra}: s block {rs:.3e}  fp block {rfp:.3e}", flush=True)


if __name__ == "__main__":
    main()
