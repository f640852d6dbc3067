/*
 * oracle.c -- CPU restatement kernels for the parity ORACLE.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product path (libpls.so) never links,
 * loads or calls it.
 *
 * What is restated here (plain C99, -ffp-contract=off so every expression
 * rounds exactly as written):
 *   - the synthetic 3-field block system of SURVEY.md 8(d) (seeded, hash based,
 *     bit-reproducible; the HIP generator in the product must match it bit for
 *     bit -- it is an input format, not the algorithm under test);
 *   - PETSc MatMult for AIJ (row-sequential dot, PetscSparseDenseDot order);
 *   - PETSc ILU(0), natural ordering, factor on the pattern of the block
 *     (MatLUFactorNumeric_SeqAIJ semantics: IKJ elimination, updates outside the
 *     pattern dropped, zero multipliers skipped, inverted diagonal stored);
 *   - PETSc MatSolve_SeqAIJ_NaturalOrdering (forward unit-lower sweep, backward
 *     upper sweep multiplying by the stored inverse diagonal).
 * PETSc itself is not in /root/reference (third-party dependency, unpinned
 * version); see oracle/__init__.py for the parity-pinning statement.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

/* ------------------------------------------------------------------ hash -- */
static inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline uint64_t hash3(uint64_t s, uint64_t a, uint64_t b) {
    return mix64(mix64(mix64(s) ^ a) ^ b);
}
static inline double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }

/* salts */
#define SALT_OFFS  0x0FF5E7ULL
#define SALT_VAL   0x5A1BE5ULL
#define SALT_DIAGA 0xD1A60AULL
#define SALT_DIAGP 0xD1A60BULL
#define SALT_BC    0x00BC00ULL
#define SALT_RHS   0x00B0B0ULL

/* ------------------------------------------------------- synthetic spec -- */
/* field ids: 0 = s (solid displacement), 1 = f (fluid velocity), 2 = p.     */
/* block ids (forward blocks, row field <= col field): ss sf sp ff fp pp.    */
enum { BSS = 0, BSF = 1, BSP = 2, BFF = 3, BFP = 4, BPP = 5 };

typedef struct {
    int dim, N;
    uint64_t seed;
    double delta;
    int64_t n[3];       /* field sizes */
    int64_t off[3];     /* field offsets in field-major order */
    int64_t W[3];       /* band per column field */
    int cnt[6];         /* offsets per forward block */
    int32_t *offs[6];   /* sorted offsets per forward block */
} synth_t;

static int blk_id(int a, int b) {
    static const int t[3][3] = {{BSS, BSF, BSP}, {BSF, BFF, BFP}, {BSP, BFP, BPP}};
    return t[a][b];
}

static int cmp_i32(const void *x, const void *y) {
    int32_t a = *(const int32_t *)x, b = *(const int32_t *)y;
    return (a > b) - (a < b);
}

/* offsets: symmetric blocks draw `half` distinct values in [1, W] and add
 * {0} and the negatives; asymmetric coupling blocks (sp, fp) draw `cnt`
 * distinct values in [-W, W].  Draw stream: mix64 chain seeded per block. */
static int draw_offsets(uint64_t seed, int bid, int symmetric, int want, int64_t W, int32_t *out) {
    uint64_t st = hash3(seed ^ SALT_OFFS, (uint64_t)bid, 0x51ULL);
    int half = symmetric ? want / 2 : want;
    int32_t *tmp = (int32_t *)malloc(sizeof(int32_t) * (size_t)(half > 0 ? half : 1));
    int got = 0;
    uint64_t range = symmetric ? (uint64_t)W : (uint64_t)(2 * W + 1);
    if ((uint64_t)half > range) { free(tmp); return -1; }
    while (got < half) {
        st = mix64(st);
        int64_t d = symmetric ? (int64_t)(1 + st % range) : (int64_t)(st % range) - W;
        int dup = 0;
        for (int k = 0; k < got; ++k) if (tmp[k] == d) { dup = 1; break; }
        if (!dup) tmp[got++] = (int32_t)d;
    }
    int m = 0;
    if (symmetric) {
        for (int k = 0; k < half; ++k) { out[m++] = tmp[k]; out[m++] = -tmp[k]; }
        out[m++] = 0;
    } else {
        for (int k = 0; k < half; ++k) out[m++] = tmp[k];
    }
    qsort(out, (size_t)m, sizeof(int32_t), cmp_i32);
    free(tmp);
    return m;
}

static int synth_init(synth_t *S, int dim, int N, uint64_t seed, double delta) {
    memset(S, 0, sizeof(*S));
    if (N < 1 || (dim != 2 && dim != 3)) return -1;
    S->dim = dim; S->N = N; S->seed = seed; S->delta = delta;
    int64_t q = 2 * (int64_t)N + 1, v = (int64_t)N + 1;
    if (dim == 3) {
        S->n[0] = S->n[1] = 3 * q * q * q; S->n[2] = v * v * v;
        S->W[0] = S->W[1] = 6 * q * q; S->W[2] = v * v + v + 1;
        int c[6] = {85, 85, 8, 85, 8, 15};
        memcpy(S->cnt, c, sizeof(c));
    } else {
        S->n[0] = S->n[1] = 2 * q * q; S->n[2] = v * v;
        S->W[0] = S->W[1] = 4 * q; S->W[2] = v + 1;
        int c[6] = {23, 23, 5, 23, 5, 7};
        memcpy(S->cnt, c, sizeof(c));
    }
    S->off[0] = 0; S->off[1] = S->n[0]; S->off[2] = S->n[0] + S->n[1];
    static const int rowf[6] = {0, 0, 0, 1, 1, 2}, colf[6] = {0, 1, 2, 1, 2, 2};
    for (int b = 0; b < 6; ++b) {
        int sym = (b == BSS || b == BSF || b == BFF || b == BPP);
        S->offs[b] = (int32_t *)malloc(sizeof(int32_t) * (size_t)S->cnt[b]);
        int m = draw_offsets(seed, b, sym, S->cnt[b], S->W[colf[b]], S->offs[b]);
        if (m != S->cnt[b]) return -2;
        (void)rowf;
    }
    return 0;
}

static void synth_free(synth_t *S) {
    for (int b = 0; b < 6; ++b) free(S->offs[b]);
}

/* ceil(m * nb / na) for the preimage of a centre value */
static inline int64_t pre_lo(int64_t m, int64_t na, int64_t nb) {
    return (m * nb + na - 1) / na;
}

/* Enumerate row `i` (local index in field a) of the full matrix in global
 * column order.  If cols != NULL writes global column ids.  Returns count.   */
static int64_t synth_row(const synth_t *S, int a, int64_t i, int64_t *cols) {
    int64_t c = 0;
    for (int b = 0; b < 3; ++b) {
        int bid = blk_id(a, b);
        const int32_t *D = S->offs[bid];
        int m = S->cnt[bid];
        int64_t na = S->n[a], nb = S->n[b];
        if (a <= b) {                    /* forward: centre + offsets */
            int64_t ctr = (a == b) ? i : (i * nb) / na;
            for (int k = 0; k < m; ++k) {
                int64_t j = ctr + D[k];
                if (j >= 0 && j < nb) { if (cols) cols[c] = S->off[b] + j; ++c; }
            }
        } else {                          /* backward: transpose of (b, a)  */
            /* rows j of field b with centre_{b->a}(j) + d == i               */
            for (int k = m - 1; k >= 0; --k) {
                int64_t mm = i - D[k];
                if (mm < 0 || mm >= na) continue;
                int64_t lo = pre_lo(mm, na, nb), hi = pre_lo(mm + 1, na, nb);
                if (hi > nb) hi = nb;
                for (int64_t j = lo; j < hi; ++j) { if (cols) cols[c] = S->off[b] + j; ++c; }
            }
        }
    }
    return c;
}

static inline int field_of(const synth_t *S, int64_t g) {
    return g < S->off[1] ? 0 : (g < S->off[2] ? 1 : 2);
}

int oracle_synth_is_bc(uint64_t seed, int64_t ip) {
    return (hash3(seed ^ SALT_BC, (uint64_t)ip, 7ULL) & 15ULL) == 0ULL;
}

/* sizes: out[0..2] = ns, nf, np;  out[3..8] = per-block offset counts */
int oracle_synth_sizes(int dim, int N, uint64_t seed, int64_t *out) {
    synth_t S;
    int rc = synth_init(&S, dim, N, seed, 0.0);
    if (rc) { synth_free(&S); return rc; }
    for (int f = 0; f < 3; ++f) out[f] = S.n[f];
    for (int b = 0; b < 6; ++b) out[3 + b] = S.cnt[b];
    synth_free(&S);
    return 0;
}

int oracle_synth_offsets(int dim, int N, uint64_t seed, int bid, int32_t *out) {
    synth_t S;
    int rc = synth_init(&S, dim, N, seed, 0.0);
    if (rc) { synth_free(&S); return rc; }
    memcpy(out, S.offs[bid], sizeof(int32_t) * (size_t)S.cnt[bid]);
    rc = S.cnt[bid];
    synth_free(&S);
    return rc;
}

/* pass 1: row counts -> row_ptr (n+1). */
int oracle_synth_rowptr(int dim, int N, uint64_t seed, int64_t *row_ptr) {
    synth_t S;
    int rc = synth_init(&S, dim, N, seed, 0.0);
    if (rc) { synth_free(&S); return rc; }
    int64_t n = S.n[0] + S.n[1] + S.n[2];
    row_ptr[0] = 0;
    /* rows are independent: the pattern does not depend on the thread count */
#pragma omp parallel for schedule(static)
    for (int64_t g = 0; g < n; ++g) {
        int a = field_of(&S, g);
        row_ptr[g + 1] = synth_row(&S, a, g - S.off[a], NULL);
    }
    for (int64_t g = 0; g < n; ++g) row_ptr[g + 1] += row_ptr[g];
    synth_free(&S);
    return 0;
}

/* pass 2: columns and values.  variant 0 = A, 1 = P, 2 = P_diff.
 * Off-diagonal (gi != gj): v = -scale * u01(hash3(seed^VAL, min, max)),
 *   scale = 1 within a field block, 0.1 across fields (B_fs = B_sf^T).
 * Diagonal: sum_{j != i} |v_ij| (sequential, column order) + delta * (1 + u),
 *   u = u01(hash3(seed^DIAG{A|P}, gi, gi)); P and P_diff use the P salt.
 * P_diff: pressure rows flagged by oracle_synth_is_bc are identity rows
 *   (pattern kept, off-diagonals zero, diagonal one) -- DirichletBC.apply.  */
int oracle_synth_fill(int dim, int N, uint64_t seed, double delta, int variant,
                      const int64_t *row_ptr, int32_t *col, double *val) {
    synth_t S;
    int rc = synth_init(&S, dim, N, seed, delta);
    if (rc) { synth_free(&S); return rc; }
    int64_t n = S.n[0] + S.n[1] + S.n[2];
    int64_t maxrow = 0;
    for (int64_t g = 0; g < n; ++g) {
        int64_t l = row_ptr[g + 1] - row_ptr[g];
        if (l > maxrow) maxrow = l;
    }
    uint64_t sv = seed ^ SALT_VAL;
    uint64_t sd = seed ^ (variant == 0 ? SALT_DIAGA : SALT_DIAGP);
    int bad = 0;
    /* rows are independent (each sums its own diagonal in column order), so
     * the values are bitwise the same for any thread count */
#pragma omp parallel reduction(| : bad)
    {
        int64_t *cols = (int64_t *)malloc(sizeof(int64_t) * (size_t)(maxrow + 1));
#pragma omp for schedule(static)
        for (int64_t g = 0; g < n; ++g) {
            int a = field_of(&S, g);
            int64_t i = g - S.off[a];
            int64_t c = synth_row(&S, a, i, cols);
            int64_t base = row_ptr[g];
            int bcrow = (variant == 2 && a == 2 && oracle_synth_is_bc(seed, i));
            double sum = 0.0;
            int64_t dpos = -1;
            for (int64_t k = 0; k < c; ++k) {
                int64_t gj = cols[k];
                col[base + k] = (int32_t)gj;
                if (gj == g) { dpos = k; val[base + k] = 0.0; continue; }
                int b = field_of(&S, gj);
                uint64_t lo = (uint64_t)(g < gj ? g : gj), hi = (uint64_t)(g < gj ? gj : g);
                double u = u01(hash3(sv, lo, hi));
                double v = (a == b) ? -u : -(0.1 * u);
                val[base + k] = bcrow ? 0.0 : v;
                sum = sum + fabs(v);
            }
            if (dpos < 0) { bad = 1; continue; }
            if (bcrow) {
                val[base + dpos] = 1.0;
            } else {
                double u = u01(hash3(sd, (uint64_t)g, (uint64_t)g));
                double sh = delta * (1.0 + u);
                val[base + dpos] = sum + sh;
            }
        }
        free(cols);
    }
    synth_free(&S);
    return bad ? -3 : 0;
}

/* right-hand side b (field-major), uniform in [-1, 1) */
void oracle_synth_rhs(uint64_t seed, int64_t n, double *b) {
    for (int64_t i = 0; i < n; ++i) {
        double u = u01(hash3(seed ^ SALT_RHS, (uint64_t)i, 3ULL));
        b[i] = 2.0 * u - 1.0;
    }
}

/* ----------------------------------------------------------- MatMult ---- */
/* y = A x (PETSc MatMult_SeqAIJ: sum = 0; sum += v[k]*x[idx[k]] in order) */
void oracle_spmv(int64_t nrows, const int64_t *rp, const int32_t *ci, const double *v,
                 const double *x, double *y, int nthreads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int64_t i = 0; i < nrows; ++i) {
        double s = 0.0;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) s = s + v[k] * x[ci[k]];
        y[i] = s;
    }
    (void)nthreads;
}

/* ------------------------------------------------------------ ILU(0) ---- */
/* In-place ILU(0) on a CSR block with sorted columns.  `lu` holds a copy of
 * the block values on entry and L (strict lower, unit diag implied), U
 * (upper incl. diagonal) on exit; `dinv[i] = 1 / u_ii` (PETSc keeps the
 * inverted pivot).  `diag[i]` = position of the diagonal in row i.
 * Returns 0, or -(i+1) for a missing diagonal, or (i+1) for a zero pivot. */
int oracle_ilu0(int64_t n, const int64_t *rp, const int32_t *ci, double *lu,
                int64_t *diag, double *dinv) {
    for (int64_t i = 0; i < n; ++i) {
        diag[i] = -1;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) if (ci[k] == i) { diag[i] = k; break; }
        if (diag[i] < 0) return (int)(-(i + 1));
    }
    /* dense work row + position map (pos[j] = index into lu or -1) */
    int64_t *pos = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    for (int64_t j = 0; j < n; ++j) pos[j] = -1;
    int rc = 0;
    for (int64_t i = 0; i < n && rc == 0; ++i) {
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) pos[ci[k]] = k;
        for (int64_t k = rp[i]; k < diag[i]; ++k) {
            int64_t r = ci[k];
            double pc = lu[k];
            if (pc != 0.0) {
                double mult = pc * dinv[r];
                lu[k] = mult;
                for (int64_t kk = diag[r] + 1; kk < rp[r + 1]; ++kk) {
                    int64_t p = pos[ci[kk]];
                    if (p >= 0) lu[p] = lu[p] - mult * lu[kk];
                }
            }
        }
        double piv = lu[diag[i]];
        if (piv == 0.0) rc = (int)(i + 1);
        else dinv[i] = 1.0 / piv;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) pos[ci[k]] = -1;
    }
    free(pos);
    return rc;
}

/* x = (LU)^{-1} b  (MatSolve_SeqAIJ_NaturalOrdering order of operations) */
void oracle_ilu0_solve(int64_t n, const int64_t *rp, const int32_t *ci, const double *lu,
                       const int64_t *diag, const double *dinv, const double *b, double *x) {
    for (int64_t i = 0; i < n; ++i) {
        double s = b[i];
        for (int64_t k = rp[i]; k < diag[i]; ++k) s = s - lu[k] * x[ci[k]];
        x[i] = s;
    }
    for (int64_t i = n - 1; i >= 0; --i) {
        double s = x[i];
        for (int64_t k = diag[i] + 1; k < rp[i + 1]; ++k) s = s - lu[k] * x[ci[k]];
        x[i] = s * dinv[i];
    }
}

/* dependency levels of the lower (dir=0) or upper (dir=1) sweep:
 * lvl[i] = 1 + max lvl[j] over the strict lower (upper) part; returns #levels */
int64_t oracle_levels(int64_t n, const int64_t *rp, const int32_t *ci, int dir, int32_t *lvl) {
    int64_t nl = 0;
    if (dir == 0) {
        for (int64_t i = 0; i < n; ++i) {
            int32_t L = 0;
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k)
                if (ci[k] < i && lvl[ci[k]] + 1 > L) L = lvl[ci[k]] + 1;
            lvl[i] = L; if (L + 1 > nl) nl = L + 1;
        }
    } else {
        for (int64_t i = n - 1; i >= 0; --i) {
            int32_t L = 0;
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k)
                if (ci[k] > i && lvl[ci[k]] + 1 > L) L = lvl[ci[k]] + 1;
            lvl[i] = L; if (L + 1 > nl) nl = L + 1;
        }
    }
    return nl;
}
