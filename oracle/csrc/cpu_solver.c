/* CPU baseline solver (TEST / MEASUREMENT INFRASTRUCTURE ONLY; see
 * oracle/__init__.py): the benchmark configuration of bench.py restated in C
 * with OpenMP -- right-preconditioned GMRES (PETSc semantics as in
 * oracle/petsc.py: classical Gram-Schmidt, Givens, restart = maxit,
 * KSPConvergedDefault, BuildSoln with the extra PC apply) with the 2-way block
 * preconditioner of lib/Preconditioner.py:219-246 and PREONLY + BJACOBI(ILU(0))
 * inner solves (PETSc block sizing, natural-ordering ILU(0) of
 * oracle.c).  SURVEY.md 8(d): "the planned CPU baseline is the build's
 * C/OpenMP restatement of the identical algorithm ... on all host cores".
 * Inner products are OpenMP reductions (their order depends on the thread
 * count), so histories agree with the Python oracle to rounding, not bitwise.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

int oracle_ilu0(int64_t n, const int64_t *rp, const int32_t *ci, double *lu, int64_t *diag, double *dinv);
void oracle_ilu0_solve(int64_t n, const int64_t *rp, const int32_t *ci, const double *lu, const int64_t *diag,
                       const double *dinv, const double *b, double *x);

#define CHUNK 2048 /* rows per cache block of the basis updates */

typedef struct {
    int64_t n, nb;
    int64_t *boff;                 /* nb + 1 block row offsets            */
    int64_t **rp, **diag;          /* per block CSR (block-local columns) */
    int32_t **ci;
    double **lu, **dinv;
} bjilu_t;

/* PCBJACOBI over rows [r0, r0 + n) x columns [c0, c0 + n) of a CSR matrix:
 * block b keeps the entries whose column falls in its own row range. */
static int bjilu_build(const int64_t *rp, const int32_t *ci, const double *v, int64_t r0, int64_t c0, int64_t n,
                       int64_t nb, bjilu_t *B) {
    if (nb > n) nb = n;
    if (nb < 1) nb = 1;
    B->n = n;
    B->nb = nb;
    B->boff = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nb + 1));
    const int64_t q = n / nb, r = n % nb;
    B->boff[0] = 0;
    for (int64_t b = 0; b < nb; ++b) B->boff[b + 1] = B->boff[b] + q + (b < r ? 1 : 0);
    B->rp = (int64_t **)calloc((size_t)nb, sizeof(int64_t *));
    B->diag = (int64_t **)calloc((size_t)nb, sizeof(int64_t *));
    B->ci = (int32_t **)calloc((size_t)nb, sizeof(int32_t *));
    B->lu = (double **)calloc((size_t)nb, sizeof(double *));
    B->dinv = (double **)calloc((size_t)nb, sizeof(double *));
    int fail = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) reduction(| : fail)
#endif
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t lo = B->boff[b], hi = B->boff[b + 1], m = hi - lo;
        int64_t cnt = 0;
        for (int64_t i = lo; i < hi; ++i)
            for (int64_t k = rp[r0 + i]; k < rp[r0 + i + 1]; ++k) {
                const int64_t c = (int64_t)ci[k] - c0;
                if (c >= lo && c < hi) ++cnt;
            }
        int64_t *brp = (int64_t *)malloc(sizeof(int64_t) * (size_t)(m + 1));
        int32_t *bci = (int32_t *)malloc(sizeof(int32_t) * (size_t)(cnt ? cnt : 1));
        double *blu = (double *)malloc(sizeof(double) * (size_t)(cnt ? cnt : 1));
        brp[0] = 0;
        int64_t p = 0;
        for (int64_t i = lo; i < hi; ++i) {
            for (int64_t k = rp[r0 + i]; k < rp[r0 + i + 1]; ++k) {
                const int64_t c = (int64_t)ci[k] - c0;
                if (c >= lo && c < hi) {
                    bci[p] = (int32_t)(c - lo);
                    blu[p] = v[k];
                    ++p;
                }
            }
            brp[i - lo + 1] = p;
        }
        B->rp[b] = brp;
        B->ci[b] = bci;
        B->lu[b] = blu;
        B->diag[b] = (int64_t *)malloc(sizeof(int64_t) * (size_t)(m ? m : 1));
        B->dinv[b] = (double *)malloc(sizeof(double) * (size_t)(m ? m : 1));
        if (oracle_ilu0(m, brp, bci, blu, B->diag[b], B->dinv[b]) != 0) fail |= 1;
    }
    return fail ? -1 : 0;
}

static void bjilu_free(bjilu_t *B) {
    for (int64_t b = 0; b < B->nb; ++b) {
        free(B->rp[b]);
        free(B->ci[b]);
        free(B->lu[b]);
        free(B->diag[b]);
        free(B->dinv[b]);
    }
    free(B->rp); free(B->ci); free(B->lu); free(B->diag); free(B->dinv); free(B->boff);
}

static void bjilu_apply(const bjilu_t *B, const double *x, double *y) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t b = 0; b < B->nb; ++b) {
        const int64_t lo = B->boff[b], m = B->boff[b + 1] - lo;
        oracle_ilu0_solve(m, B->rp[b], B->ci[b], B->lu[b], B->diag[b], B->dinv[b], x + lo, y + lo);
    }
}

/* y = z - M x over rows [r0, r0+m) and columns [0, nc) of a CSR matrix */
static void spmv_rows(const int64_t *rp, const int32_t *ci, const double *v, int64_t r0, int64_t m, int64_t nc,
                      const double *x, const double *z, double *y) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t i = 0; i < m; ++i) {
        double s = 0.0;
        for (int64_t k = rp[r0 + i]; k < rp[r0 + i + 1]; ++k)
            if (ci[k] < nc) s += v[k] * x[ci[k]];
        y[i] = z ? z[i] - s : s;
    }
}

/* fixed-order dot: 64 contiguous chunks summed left to right, then the chunk
 * sums in order -- the same value for any thread count and any run (an
 * OpenMP reduction combines the threads' partials in completion order, which
 * moved GMRES's crossing of rtol by several iterations between runs) */
static double dot(int64_t n, const double *a, const double *b) {
    enum { NCH = 64 };
    double part[NCH];
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int c = 0; c < NCH; ++c) {
        const int64_t lo = n * c / NCH, hi = n * (c + 1) / NCH;
        double s = 0.0;
        for (int64_t i = lo; i < hi; ++i) s += a[i] * b[i];
        part[c] = s;
    }
    double s = 0.0;
    for (int c = 0; c < NCH; ++c) s += part[c];
    return s;
}

typedef struct {
    const int64_t *Arp, *Prp;
    const int32_t *Aci, *Pci;
    const double *Av, *Pv;
    int64_t n, ns;
    bjilu_t Ks, Kfp;
    double *t;
} blockpc_t;

/* y = M^-1 x: y_s = Ks^-1 x_s ; y_fp = Kfp^-1 (x_fp - P_fp,s y_s) */
static void pc_apply(blockpc_t *M, const double *x, double *y) {
    const int64_t ns = M->ns, nfp = M->n - ns;
    bjilu_apply(&M->Ks, x, y);
    spmv_rows(M->Prp, M->Pci, M->Pv, ns, nfp, ns, y, x + ns, M->t);
    bjilu_apply(&M->Kfp, M->t, y + ns);
}

/* Returns iterations; *reason = PETSc KSPConvergedReason; hist[0..its]. */
int cpu_gmres_2way(int64_t n, int64_t ns, const int64_t *Arp, const int32_t *Aci, const double *Av,
                   const int64_t *Prp, const int32_t *Pci, const double *Pv, int64_t nb_s, int64_t nb_fp,
                   double rtol, double atol, int maxit, const double *b, double *x, int *reason, double *hist,
                   int nthreads, double *t_setup, double *t_solve) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
    double t0 = omp_get_wtime();
#else
    (void)nthreads;
    double t0 = 0;
#endif
    blockpc_t M = {Arp, Prp, Aci, Pci, Av, Pv, n, ns, {0}, {0}, NULL};
    if (bjilu_build(Prp, Pci, Pv, 0, 0, ns, nb_s, &M.Ks) || bjilu_build(Prp, Pci, Pv, ns, ns, n - ns, nb_fp, &M.Kfp))
        return -1;
    M.t = (double *)malloc(sizeof(double) * (size_t)(n - ns));
#ifdef _OPENMP
    double t1 = omp_get_wtime();
#else
    double t1 = 0;
#endif
    const int mk = maxit;
    double *V = (double *)malloc(sizeof(double) * (size_t)n * (size_t)(mk + 1));
    double *w = (double *)malloc(sizeof(double) * (size_t)n);
    double *tmp = (double *)malloc(sizeof(double) * (size_t)n);
    double *HH = (double *)calloc((size_t)(mk + 1) * (size_t)(mk + 1), sizeof(double));
    double *cc = (double *)calloc((size_t)mk + 1, sizeof(double)), *ss = (double *)calloc((size_t)mk + 1, sizeof(double));
    double *grs = (double *)calloc((size_t)mk + 2, sizeof(double)), *h = (double *)calloc((size_t)mk + 1, sizeof(double));
#define H_(i, j) HH[(size_t)(i) * (size_t)(mk + 1) + (size_t)(j)]
    memset(x, 0, sizeof(double) * (size_t)n);
    int its = 0;
    *reason = 0;
    /* single cycle (restart = maxit): r0 = b */
    double res = sqrt(dot(n, b, b));
    hist[0] = res;
    const double ttol = fmax(rtol * res, atol);
    if (res == 0.0) {
        *reason = 3;
    } else if (res <= ttol) {
        *reason = res < atol ? 3 : 2;
    }
    if (!*reason) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
        for (int64_t i = 0; i < n; ++i) V[i] = b[i] * (1.0 / res);
        grs[0] = res;
        int loc = 0;
        while (!*reason && loc < mk && its < maxit) {
            double *vk = V + (size_t)loc * (size_t)n, *vn = V + (size_t)(loc + 1) * (size_t)n;
            pc_apply(&M, vk, tmp);
            spmv_rows(Arp, Aci, Av, 0, n, n, tmp, NULL, w);
            for (int j = 0; j <= loc; ++j) h[j] = dot(n, V + (size_t)j * (size_t)n, w);
            /* w -= sum_j h_j V_j (j ascending), cache-blocked over rows */
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
            for (int64_t i0 = 0; i0 < n; i0 += CHUNK) {
                const int64_t i1 = i0 + CHUNK < n ? i0 + CHUNK : n;
                for (int j = 0; j <= loc; ++j) {
                    const double hj = h[j], *vj = V + (size_t)j * (size_t)n;
                    for (int64_t i = i0; i < i1; ++i) w[i] -= hj * vj[i];
                }
            }
            for (int j = 0; j <= loc; ++j) H_(j, loc) = h[j];
            const double tt = sqrt(dot(n, w, w));
            H_(loc + 1, loc) = tt;
            double hapbnd = fabs(tt / grs[loc]);
            if (hapbnd > 1e-30) hapbnd = 1e-30;
            const int hapend = tt < hapbnd;
            if (!hapend) {
                const double inv = 1.0 / tt;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
                for (int64_t i = 0; i < n; ++i) vn[i] = w[i] * inv;
            }
            for (int j = 0; j < loc; ++j) {
                const double t0j = H_(j, loc);
                H_(j, loc) = cc[j] * t0j + ss[j] * H_(j + 1, loc);
                H_(j + 1, loc) = cc[j] * H_(j + 1, loc) - ss[j] * t0j;
            }
            if (!hapend) {
                const double tg = sqrt(H_(loc, loc) * H_(loc, loc) + H_(loc + 1, loc) * H_(loc + 1, loc));
                if (tg == 0.0) { *reason = -2; break; }
                cc[loc] = H_(loc, loc) / tg;
                ss[loc] = H_(loc + 1, loc) / tg;
                grs[loc + 1] = -(ss[loc] * grs[loc]);
                grs[loc] = cc[loc] * grs[loc];
                H_(loc, loc) = cc[loc] * H_(loc, loc) + ss[loc] * H_(loc + 1, loc);
                res = fabs(grs[loc + 1]);
            } else {
                res = 0.0;
            }
            ++loc;
            ++its;
            hist[its] = res;
            if (isnan(res) || isinf(res)) *reason = -9;
            else if (res <= ttol) *reason = res < atol ? 3 : 2;
            else if (hapend) *reason = -5;
        }
        /* BuildSoln: back substitution, tmp = V y, x = M^-1 tmp */
        const int it = loc - 1;
        if (it >= 0 && H_(it, it) != 0.0) {
            double *nrs = (double *)calloc((size_t)it + 1, sizeof(double));
            nrs[it] = grs[it] / H_(it, it);
            for (int k = it - 1; k >= 0; --k) {
                double t0k = grs[k];
                for (int j = k + 1; j <= it; ++j) t0k -= H_(k, j) * nrs[j];
                nrs[k] = t0k / H_(k, k);
            }
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
            for (int64_t i0 = 0; i0 < n; i0 += CHUNK) {
                const int64_t i1 = i0 + CHUNK < n ? i0 + CHUNK : n;
                for (int64_t i = i0; i < i1; ++i) tmp[i] = 0.0;
                for (int j = 0; j <= it; ++j) {
                    const double c = nrs[j], *vj = V + (size_t)j * (size_t)n;
                    for (int64_t i = i0; i < i1; ++i) tmp[i] += c * vj[i];
                }
            }
            pc_apply(&M, tmp, x);
            free(nrs);
        }
        if (!*reason && its >= maxit) *reason = -3;
    }
#undef H_
#ifdef _OPENMP
    double t2 = omp_get_wtime();
#else
    double t2 = 0;
#endif
    *t_setup = t1 - t0;
    *t_solve = t2 - t1;
    free(V); free(w); free(tmp); free(HH); free(cc); free(ss); free(grs); free(h); free(M.t);
    bjilu_free(&M.Ks);
    bjilu_free(&M.Kfp);
    return its;
}
