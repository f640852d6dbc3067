"""Check: the device's synthetic right-hand side (pls_synthetic_rhs_device) equals
the oracle's S.rhs for the same seed, and the CPU port's iteration count on it
equals the device's (bench.py's cpu_baseline premise).  usage: rhs_check.py N [nb_s nb_fp]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "poroelasticity-linear-solvers_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402


def main():
    N = int(sys.argv[1])
    nb_s, nb_fp = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (64, 64)
    import lib._native as Nt
    from lib.handle import Handle
    from oracle import native
    from oracle import synthetic as S
    from test_gpu_large import _opts
    SEED, DELTA, RHS = 20261015, 0.05, 7
    spec = S.SynthSpec(3, N, SEED, DELTA)
    h = Handle.synthetic(3, N, SEED, DELTA, _opts(nb_s, nb_fp))
    n = h.n
    d_b, d_x = Nt.DeviceArray(n), Nt.DeviceArray(n)
    h.rhs_device(RHS, d_b.p)
    bd = d_b.download()
    perm = h.permutation() if hasattr(h, "permutation") else None
    bo = S.rhs(S.SynthSpec(3, N, RHS, DELTA))
    print("n", n, "oracle n", bo.size, "equal", bool(np.array_equal(bd, bo)), flush=True)
    if perm is not None:
        print("perm identity", bool(np.array_equal(np.asarray(perm), np.arange(n))), flush=True)
    res = h.solve_device(d_b.p, d_x.p)
    A, P = S.matrix(spec, 0), S.matrix(spec, 1)
    ns = spec.sizes()[0]
    for name, b in (("oracle rhs", bo), ("device rhs", bd)):
        _, its, reason, _, _, _ = native.cpu_gmres_2way(A, P, ns, nb_s, nb_fp, b, rtol=1e-6, atol=1e-8, maxit=100,
                                                      nthreads=16)
        print(name, "cpu its", its, "device its", res.its, flush=True)


if __name__ == "__main__":
    main()
