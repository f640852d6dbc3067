"""SpMV of an assembled swelling system under SpMV layout variants (GPU).

usage: python tools/spmv_fe.py <dim> <N> [key=value,key=value ...]...
Assembles lib/fe_swelling once (2-way internal order), builds one handle per
variant (library options, e.g. pls.d16_sigma=0), and prints one JSON line per
variant: layout bytes, CSR-algorithmic bytes, isolated
y = A x launch time (HIP events, 20 launches), GB/s of both.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poroelasticity-linear-solvers_amd")]

import numpy as np  # noqa: E402


def main():
    dim, N = int(sys.argv[1]), int(sys.argv[2])
    variants = [dict(kv.split("=", 1) for kv in v.split(",") if kv) for v in (sys.argv[3:] or [""])]
    import lib._native as Nt
    from lib.fe_swelling import assemble_swelling
    from lib.handle import Handle
    Nt.check(Nt.lib().pls_set_device(0))
    t0 = time.perf_counter()
    s = assemble_swelling(dim, N, "diagonal")
    print(f"[spmv_fe] assembled {dim}-D N={N}: n={s.A.shape[0]} nnz={s.A.nnz} in {time.perf_counter() - t0:.1f}s",
          file=sys.stderr, flush=True)
    n, nnz = s.A.shape[0], s.A.nnz
    alg = 12.0 * nnz + 8.0 * (n + 1) + 16.0 * n
    x = np.random.default_rng(1).standard_normal(n)
    ref = s.A @ x
    base = {"pls.pc_type": "diagonal", "s_pc_type": "jacobi", "fp_pc_type": "jacobi", "pls.inner_pc_type": "jacobi",
            "pls.inner_ksp_type": "preonly"}
    for v in variants:
        h = Handle.from_csr(s.A, s.P, None, s.is_s, s.is_f, s.is_p, [], dict(base, **v))
        y = h.matmult(x)
        err = float(np.max(np.abs(y - ref) / (abs(s.A) @ np.abs(x))))
        h.create_solver()
        dx, dy = Nt.DeviceArray(n), Nt.DeviceArray(n)
        dx.upload(x)
        sec = h.bench_spmv(dx.p, dy.p, 20)
        d16, mb = h.spmv_layout()
        lay = mb + 16.0 * n
        print(json.dumps({"variant": v, "n": n, "nnz": nnz, "d16": d16, "layout_bytes": lay, "alg_bytes": alg,
                          "layout_over_alg": lay / alg, "us": sec * 1e6, "alg_gbs": alg / sec / 1e9,
                          "frac": alg / sec / 8e12, "layout_gbs": lay / sec / 1e9, "max_rel_err": err}), flush=True)
        dx.free()
        dy.free()
        h.destroy()


if __name__ == "__main__":
    main()
