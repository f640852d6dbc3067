// dense.hip -- exact LU (PCLU) of small field blocks as a dense inverse.
//
// The reference's exact option set factors every field block with MUMPS
// (petsc-options-exact:11-35, PREONLY + LU): y = K^-1 x up to rounding.  A
// level-scheduled sparse LU on the envelope pattern is a chain of n dependent
// rows (every row of a banded or arrow-shaped profile depends on the one
// before it), which is launch- and latency-bound far below HBM speed.  For
// blocks up to a few 10^4 rows the device instead forms K^-1 once by blocked
// Gauss-Jordan elimination (no pivoting, as the sparse path; 2 n^3 flops on
// 64 x 64 LDS tiles) and every application is one HBM-bound dense GEMV
// (8 n^2 bytes).  Storage: row-major, leading dimension ld = 64 * ceil(n/64),
// padding rows/columns are identity rows/columns (they never couple).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace pls {

static constexpr int DB = 64;    // block size
static constexpr int DTPB = 256; // threads per tile workgroup (16 x 16, 4 x 4 outputs each)

// M = 0 with identity padding, then scatter the CSR rows.
__global__ __launch_bounds__(256) void k_dense_pad(int64_t n, int64_t ld, double *M) {
    const int64_t i = n + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < ld) M[i * ld + i] = 1.0;
}
__global__ __launch_bounds__(256) void k_dense_scatter(int64_t n, int64_t ld, const int64_t *rp, const int32_t *ci,
                                                       const double *val, double *M) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    for (int64_t k = rp[i] + (threadIdx.x & 63); k < rp[i + 1]; k += 64) M[i * ld + ci[k]] = val[k];
}
void launch_dense_from_csr(int64_t n, int64_t ld, const int64_t *rp, const int32_t *ci, const double *val, double *M,
                           hipStream_t st) {
    (void)hipMemsetAsync(M, 0, sizeof(double) * (size_t)ld * ld, st);
    if (ld > n) k_dense_pad<<<(unsigned)((ld - n + 255) / 256), 256, 0, st>>>(n, ld, M);
    if (n > 0) k_dense_scatter<<<(unsigned)((n + 3) / 4), 256, 0, st>>>(n, ld, rp, ci, val, M);
}

// In-place Gauss-Jordan inverse of the diagonal block M_kk (one workgroup):
// D = M_kk^-1 written to D (64 x 64, row-major).  fail |= 1 on a zero pivot.
#pragma clang fp contract(off)
__global__ __launch_bounds__(DTPB) void k_gj_diag(int64_t ld, int64_t k, const double *M, double *D, int32_t *fail) {
    __shared__ double a[DB][DB + 1];
    const double *src = M + (k * DB) * ld + k * DB;
    for (int t = threadIdx.x; t < DB * DB; t += DTPB) a[t / DB][t % DB] = src[(int64_t)(t / DB) * ld + t % DB];
    __syncthreads();
    for (int p = 0; p < DB; ++p) {
        const double piv = a[p][p];
        __syncthreads();
        if (piv == 0.0) {
            if (threadIdx.x == 0) atomicOr(fail, 1);
            return;  // uniform across the workgroup
        }
        // pivot row: a[p][j] /= piv (a[p][p] := 1 / piv)
        if (threadIdx.x < DB) {
            const int j = threadIdx.x;
            a[p][j] = (j == p) ? 1.0 / piv : a[p][j] / piv;
        }
        __syncthreads();
        // other rows: a[i][j] -= a[i][p] a[p][j]; a[i][p] := -a[i][p] / piv
        double f[DB * DB / DTPB];
        for (int u = 0; u < DB * DB / DTPB; ++u) {
            const int t = threadIdx.x + u * DTPB;
            f[u] = a[t / DB][p];
        }
        __syncthreads();
        for (int u = 0; u < DB * DB / DTPB; ++u) {
            const int t = threadIdx.x + u * DTPB, i = t / DB, j = t % DB;
            if (i == p) continue;
            if (j == p) a[i][j] = -f[u] * a[p][p];
            else a[i][j] = a[i][j] - f[u] * a[p][j];
        }
        __syncthreads();
    }
    for (int t = threadIdx.x; t < DB * DB; t += DTPB) D[t] = a[t / DB][t % DB];
}
#pragma clang fp contract(on)

// ---------------------------------------------- threshold partial pivoting --
// MUMPS's pivot rule (CNTL(1) = u, 0.01 for unsymmetric matrices) before the
// Gauss-Jordan step k of a front (or of the dense block): the 64 pivots of tile
// column k are chosen among the front's remaining fully-summed rows [r0, r0 + m)
// -- not only the tile's own 64 -- by an LU with threshold partial pivoting of
// that panel (a scratch copy P, with the q update rows below it as the
// threshold's reference: they are eliminated too but never chosen): column j
// keeps its diagonal row while |a_jj| >= u max_i |a_ij| over the candidates,
// else takes the largest (ties: the smaller row).  The chosen rows are then
// swapped into the tile's positions in W -- whole rows, every column -- and in
// rowperm (front-local original row of each position), so the elimination
// that follows factors Pi F; the solves permute the right-hand side alike.
// stats[0]: rows exchanged, [1]: pivots below u x the column's largest entry
// over the candidates and the update rows (the pivots MUMPS would delay to the
// parent; here the best candidate is used), [2]: columns with no nonzero
// candidate (singular fully-summed block).
__device__ void panel_pivot(double *W, int64_t ld, int64_t r0, int m, int64_t ur0, int q, double *P,
                            int32_t *rowperm, int32_t *stats, double u, int32_t *dflag = nullptr) {
    __shared__ double rv[DTPB], rc[DTPB];
    __shared__ int ri[DTPB];
    __shared__ int swp[DB];
    const int tid = threadIdx.x;
    const int nr = m + q, nc = m < DB ? m : DB;
    for (int64_t t = tid; t < (int64_t)nr * DB; t += DTPB) {
        const int64_t i = t >> 6, c = t & 63;
        const int64_t row = i < m ? r0 + i : ur0 + (i - m);
        P[t] = W[row * ld + r0 + c];
    }
    __syncthreads();
    for (int j = 0; j < nc; ++j) {
        double bv = -1.0, cv = 0.0;
        int bi = m;
        for (int i = j + tid; i < m; i += DTPB) {  // ascending per thread: a tie keeps the smaller row
            const double v = fabs(P[(int64_t)i * DB + j]);
            if (v > bv) {
                bv = v;
                bi = i;
            }
        }
        for (int i = m + tid; i < nr; i += DTPB) cv = fmax(cv, fabs(P[(int64_t)i * DB + j]));
        rv[tid] = bv;
        ri[tid] = bi;
        rc[tid] = cv;
        __syncthreads();
        for (int o = DTPB / 2; o > 0; o >>= 1) {
            if (tid < o) {
                const double v2 = rv[tid + o];
                const int i2 = ri[tid + o];
                if (v2 > rv[tid] || (v2 == rv[tid] && i2 < ri[tid])) {
                    rv[tid] = v2;
                    ri[tid] = i2;
                }
                rc[tid] = fmax(rc[tid], rc[tid + o]);
            }
            __syncthreads();
        }
        if (tid == 0) {
            const double amax = rv[0], dj = fabs(P[(int64_t)j * DB + j]);
            const int sel = (amax > 0.0 && dj < u * amax) ? ri[0] : j;
            if (sel != j) atomicAdd(stats, 1);
            if (amax < u * fmax(amax, rc[0])) {
                atomicAdd(stats + 1, 1);
                if (dflag) dflag[r0 + j] = 1;  // column (unknown) r0 + j of the front: MUMPS would delay it
            }
            if (amax == 0.0) atomicAdd(stats + 2, 1);
            swp[j] = sel;
        }
        __syncthreads();
        const int sel = swp[j];
        if (sel != j && tid < DB) {
            const double t0 = P[(int64_t)j * DB + tid];
            P[(int64_t)j * DB + tid] = P[(int64_t)sel * DB + tid];
            P[(int64_t)sel * DB + tid] = t0;
        }
        __syncthreads();
        const double d = P[(int64_t)j * DB + j];
        if (d != 0.0)
            for (int i = j + 1 + tid; i < nr; i += DTPB) {
                double *pi = P + (int64_t)i * DB;
                const double l = pi[j] / d;
                pi[j] = l;
                for (int c = j + 1; c < DB; ++c) pi[c] = pi[c] - l * P[(int64_t)j * DB + c];
            }
        __syncthreads();
    }
    for (int j = 0; j < nc; ++j) {  // the exchanges, in order, on whole rows of W
        const int sel = swp[j];
        if (sel == j) continue;
        double *a = W + (r0 + j) * ld, *b = W + (r0 + sel) * ld;
        for (int64_t c = tid; c < ld; c += DTPB) {
            const double t0 = a[c];
            a[c] = b[c];
            b[c] = t0;
        }
        if (tid == 0) {
            const int32_t t0 = rowperm[r0 + j];
            rowperm[r0 + j] = rowperm[r0 + sel];
            rowperm[r0 + sel] = t0;
        }
        __syncthreads();
    }
}

// The panel's common case, in parallel: the diagonal row kept in every column.
// Then the panel's elimination is the unpivoted one, a_ij at step j is l_ij u_jj
// with L = A U11^-1 (U11: the tile's unpivoted LU), and the rule above reads
//   exchange in column j   <=>  u x max_{candidates i > j} |l_ij| > 1,
//   below u x column max   <=>  max(1, max_cand |l_ij|) < u x max_{update rows} |l_ij|.
// k_panel_tile (one workgroup per panel) factors the tile, k_panel_rows (a
// thread per row below it, many workgroups) forms the rows of L by the same
// right-looking updates as panel_pivot and takes the column maxima; the
// per-panel workgroup (k_*_panel_pivot) then sets the statistics and the delay
// flags from them, or -- on an exchange, a zero or a non-finite entry -- runs
// panel_pivot itself.  Rounds 1-6's one-workgroup panel alone took ~23 s of
// the 30 s setup at footing N = 80 (inexact; a 29,988-row dense block), with
// no exchange at all.
// Per-panel scratch (PANEL_FAST doubles): U11 [64][64], then the column maxima
// of |l| over candidates (64) and update rows (64) as the bits of non-negative
// doubles (ordered as unsigned integers), then a flag (bad entry).
static constexpr int PANEL_FAST = 4096 + 192;
struct PanelRef {
    double *W;
    int64_t ld, r0, ur0;
    int m, q;  // candidates [r0, r0 + m), update rows [ur0, ur0 + q)
};
__device__ __forceinline__ bool mf_panel_ref(const MFront &f, int k, double *W, PanelRef &p) {
    p.r0 = (int64_t)k * DB;
    // nothing to choose and nothing to compare with: every candidate is in the tile, whose own
    // partial pivoting (k_mf_gj_diag) takes the same rows, and no update rows
    if (k >= f.pt || p.r0 >= f.p || (f.p - p.r0 <= DB && f.q == 0)) return false;
    p.W = W + f.ws;
    p.ld = (int64_t)f.ldt * DB;
    p.ur0 = (int64_t)f.pt * DB;
    p.m = (int)(f.p - p.r0);
    p.q = f.q;
    return true;
}
__device__ __forceinline__ bool dense_panel_ref(int64_t n, int64_t ld, int64_t k, double *M, PanelRef &p) {
    p.r0 = k * DB;
    if (p.r0 >= n) return false;
    p.W = M;
    p.ld = ld;
    p.ur0 = 0;
    p.m = (int)(n - p.r0);
    p.q = 0;
    return true;
}
__device__ __forceinline__ const double *panel_row(const PanelRef &p, int i) {  // panel row i, column r0
    return p.W + (i < p.m ? p.r0 + i : p.ur0 + (i - p.m)) * p.ld + p.r0;
}
__device__ __forceinline__ uint64_t dbits(double v) { return (uint64_t)__double_as_longlong(v); }

__device__ void panel_tile(const PanelRef &p, double *S) {
    __shared__ double T[DB][DB + 1];
    __shared__ int sbad;
    const int tid = threadIdx.x, nc = p.m < DB ? p.m : DB;
    if (tid == 0) sbad = 0;
    for (int t = tid; t < DB * DB; t += DTPB) {
        const int i = t >> 6, c = t & 63;
        T[i][c] = i < nc ? panel_row(p, i)[c] : 0.0;
    }
    __syncthreads();
    const int i = tid >> 2, c0 = (tid & 3) * 16;  // row i, columns [c0, c0 + 16)
    bool bad = false;
    for (int j = 0; j < nc; ++j) {
        const double d = T[j][j];
        bad = bad || d == 0.0 || !(fabs(d) <= 1.7976931348623157e308);
        const double l = (i > j && i < nc) ? T[i][j] / d : 0.0;
        __syncthreads();
        if (i > j && i < nc) {
            for (int c = c0 > j + 1 ? c0 : j + 1; c < c0 + 16; ++c) T[i][c] = T[i][c] - l * T[j][c];
            if (c0 == 0) T[i][j] = l;
        }
        __syncthreads();
    }
    for (int t = tid; t < DB * DB; t += DTPB) S[t] = T[t >> 6][t & 63];
    uint64_t *mx = reinterpret_cast<uint64_t *>(S + 4096);
    if (tid < DB) {
        double mc = 0.0;
        for (int r = tid + 1; r < nc; ++r) mc = fmax(mc, fabs(T[r][tid]));
        if (!(mc <= 1.7976931348623157e308)) bad = true;
        mx[tid] = dbits(mc);
        mx[64 + tid] = 0;
    }
    if (bad) sbad = 1;
    __syncthreads();
    if (tid == 0) mx[128] = sbad;
}
static constexpr int PRTPB = 128;  // k_panel_rows: rows per workgroup (a thread each; LDS: the rows + U11)
__device__ void panel_rows(const PanelRef &p, const double *S) {
    __shared__ double U[DB][DB + 1];
    __shared__ double A[DB][PRTPB];  // A[c][t]: column c of the workgroup's row t
    const int tid = threadIdx.x, lane = tid & 63, nc = p.m < DB ? p.m : DB;
    const int i0 = nc + (int)blockIdx.x * PRTPB, nr = p.m + p.q;
    for (int t = tid; t < DB * DB; t += PRTPB) U[t >> 6][t & 63] = S[t];
    for (int t = tid; t < DB * PRTPB; t += PRTPB) {  // (coalesced: 64 threads per row)
        const int r = t >> 6, c = t & 63;
        A[c][r] = i0 + r < nr && c < nc ? panel_row(p, i0 + r)[c] : 0.0;
    }
    __syncthreads();
    const int i = i0 + tid;  // panel row (below the tile)
    const bool act = i < nr;
    bool bad = false;
    uint64_t *mx = reinterpret_cast<uint64_t *>(const_cast<double *>(S) + 4096);
    uint64_t myc = 0, myu = 0;
    // the right-looking updates of panel_pivot, row by row: bitwise its l
    for (int j = 0; j < nc; ++j) {
        const double l = A[j][tid] / U[j][j];
        for (int c = j + 1; c < DB; ++c) A[c][tid] = A[c][tid] - l * U[j][c];
        const double al = act ? fabs(l) : 0.0;
        bad = bad || !(al <= 1.7976931348623157e308);
        double vc = i < p.m ? al : 0.0, vu = i < p.m ? 0.0 : al;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            vc = fmax(vc, __shfl_xor(vc, o));
            vu = fmax(vu, __shfl_xor(vu, o));
        }
        if (lane == j) {
            myc = dbits(vc);
            myu = dbits(vu);
        }
    }
    if (lane < nc) {
        if (myc) atomicMax(reinterpret_cast<unsigned long long *>(mx + lane), (unsigned long long)myc);
        if (myu) atomicMax(reinterpret_cast<unsigned long long *>(mx + 64 + lane), (unsigned long long)myu);
    }
    if (bad) atomicMax(reinterpret_cast<unsigned long long *>(mx + 128), 1ull);
}
// true: the fast path holds for this panel (statistics and flags set)
__device__ bool panel_fast_done(const PanelRef &p, const double *S, int32_t *stats, double u, int32_t *dflag) {
    __shared__ int slow;
    const int tid = threadIdx.x, nc = p.m < DB ? p.m : DB;
    const uint64_t *mx = reinterpret_cast<const uint64_t *>(S + 4096);
    if (tid == 0) slow = mx[128] != 0;
    __syncthreads();
    if (tid < nc && u * __longlong_as_double((long long)mx[tid]) > 1.0) slow = 1;
    __syncthreads();
    const bool s = slow;
    __syncthreads();  // (slow is read by every thread before the next panel's use)
    if (s) return false;
    if (tid < nc) {
        const double mc = __longlong_as_double((long long)mx[tid]), mu = __longlong_as_double((long long)mx[64 + tid]);
        if (fmax(1.0, mc) < u * mu) {
            atomicAdd(stats + 1, 1);
            if (dflag) dflag[p.r0 + tid] = 1;
        }
    }
    return true;
}

template <bool MF>
__global__ __launch_bounds__(DTPB) void k_panel_tile(const MFront *F, int64_t n, int64_t ld, int k, double *W,
                                                     double *S) {
    PanelRef p;
    if (!(MF ? mf_panel_ref(F[blockIdx.x], k, W, p) : dense_panel_ref(n, ld, k, W, p))) return;
    panel_tile(p, S + (int64_t)blockIdx.x * PANEL_FAST);
}
template <bool MF>
__global__ __launch_bounds__(PRTPB) void k_panel_rows(const MFront *F, int64_t n, int64_t ld, int k, double *W,
                                                      double *S) {
    PanelRef p;
    if (!(MF ? mf_panel_ref(F[blockIdx.y], k, W, p) : dense_panel_ref(n, ld, k, W, p))) return;
    const int nc = p.m < DB ? p.m : DB;
    if (nc + (int64_t)blockIdx.x * PRTPB >= p.m + p.q) return;  // (uniform: no row of this panel here)
    panel_rows(p, S + (int64_t)blockIdx.y * PANEL_FAST);
}

// dense block (PCDenseLU): candidates rows [64 k, n), no update rows
__global__ __launch_bounds__(DTPB) void k_dense_panel_pivot(int64_t n, int64_t ld, int64_t k, double *M, double *P,
                                                            int32_t *rowperm, int32_t *stats, double u,
                                                            const double *S) {
    PanelRef p;
    if (!dense_panel_ref(n, ld, k, M, p)) return;
    if (S && panel_fast_done(p, S, stats, u, nullptr)) return;
    panel_pivot(M, ld, p.r0, p.m, 0, 0, P, rowperm, stats, u);
}
// fronts (blockIdx.x): candidates rows [64 k, p), update rows [64 pt, 64 pt + q);
// P + soff[f]: (p + q) x 64 scratch; rowperm + pst[f]: the front's pivot rows
static constexpr int PANEL_LDS_ROWS = 160;  // panels of up to this many rows stay in LDS (80 KiB)
__global__ __launch_bounds__(DTPB) void k_mf_panel_pivot(const MFront *F, const int64_t *pst, const int64_t *soff,
                                                         int k, double *W, double *P, int32_t *rowperm,
                                                         int32_t *stats, double u, int32_t *dflag, const double *S) {
    __shared__ double Pl[PANEL_LDS_ROWS * DB];
    PanelRef p;
    if (!mf_panel_ref(F[blockIdx.x], k, W, p)) return;
    int32_t *df = dflag ? dflag + pst[blockIdx.x] : nullptr;
    if (S && panel_fast_done(p, S + (int64_t)blockIdx.x * PANEL_FAST, stats, u, df)) return;
    const int nr = p.m + p.q;
    panel_pivot(p.W, p.ld, p.r0, p.m, p.ur0, p.q, nr <= PANEL_LDS_ROWS ? Pl : P + soff[blockIdx.x],
                rowperm + pst[blockIdx.x], stats, u, df);
}

// C (64 x 64 tile, leading dimension ld) := alpha * op: tile-by-tile products
// with 4 x 4 outputs per thread; A^T staged in LDS so the A reads broadcast.
__device__ __forceinline__ void tile_load(const double *src, int64_t ld, double (*dst)[DB + 1], bool transpose) {
    for (int t = threadIdx.x; t < DB * DB; t += DTPB) {
        const int r = t / DB, cc = t % DB;
        const double v = src[(int64_t)r * ld + cc];
        if (transpose) dst[cc][r] = v; else dst[r][cc] = v;
    }
}

// Row panel: M_kj := D M_kj for every block column j != k (blockIdx.x = j'),
// and M_kk := D (blockIdx.x == k).
__global__ __launch_bounds__(DTPB) void k_gj_rowpanel(int64_t ld, int64_t k, const double *D, double *M) {
    __shared__ double at[DB][DB + 1];  // D^T
    __shared__ double b[DB][DB + 1];
    const int64_t j = blockIdx.x;
    double *C = M + (k * DB) * ld + j * DB;
    if (j == k) {
        for (int t = threadIdx.x; t < DB * DB; t += DTPB) C[(int64_t)(t / DB) * ld + t % DB] = D[t];
        return;
    }
    tile_load(D, DB, at, true);
    tile_load(C, ld, b, false);
    __syncthreads();
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    double acc[4][4] = {};
    for (int kk = 0; kk < DB; ++kk) {
        double av[4], bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) av[r] = at[kk][ty + 16 * r];
#pragma unroll
        for (int q = 0; q < 4; ++q) bv[q] = b[kk][tx + 16 * q];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] += av[r] * bv[q];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) C[(int64_t)(ty + 16 * r) * ld + tx + 16 * q] = acc[r][q];
}

// Update: M_ij -= M_ik M_kj for i != k, j != k (blockIdx = (j', i') skipping k).
__global__ __launch_bounds__(DTPB) void k_gj_update(int64_t ld, int64_t k, double *M) {
    __shared__ double at[DB][DB + 1];  // M_ik^T
    __shared__ double b[DB][DB + 1];   // M_kj
    const int64_t j = blockIdx.x + (blockIdx.x >= k ? 1 : 0);
    const int64_t i = blockIdx.y + (blockIdx.y >= k ? 1 : 0);
    tile_load(M + (i * DB) * ld + k * DB, ld, at, true);
    tile_load(M + (k * DB) * ld + j * DB, ld, b, false);
    __syncthreads();
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    double acc[4][4] = {};
    for (int kk = 0; kk < DB; ++kk) {
        double av[4], bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) av[r] = at[kk][ty + 16 * r];
#pragma unroll
        for (int q = 0; q < 4; ++q) bv[q] = b[kk][tx + 16 * q];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] += av[r] * bv[q];
    }
    double *C = M + (i * DB) * ld + j * DB;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double *c = C + (int64_t)(ty + 16 * r) * ld + tx + 16 * q;
            *c = *c - acc[r][q];
        }
}

// Column panel: M_ik := -M_ik D for i != k (blockIdx.x = i' skipping k).
__global__ __launch_bounds__(DTPB) void k_gj_colpanel(int64_t ld, int64_t k, const double *D, double *M) {
    __shared__ double at[DB][DB + 1];  // M_ik^T
    __shared__ double b[DB][DB + 1];   // D
    const int64_t i = blockIdx.x + (blockIdx.x >= k ? 1 : 0);
    double *C = M + (i * DB) * ld + k * DB;
    tile_load(C, ld, at, true);
    tile_load(D, DB, b, false);
    __syncthreads();
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    double acc[4][4] = {};
    for (int kk = 0; kk < DB; ++kk) {
        double av[4], bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) av[r] = at[kk][ty + 16 * r];
#pragma unroll
        for (int q = 0; q < 4; ++q) bv[q] = b[kk][tx + 16 * q];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] += av[r] * bv[q];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) C[(int64_t)(ty + 16 * r) * ld + tx + 16 * q] = -acc[r][q];
}

void launch_dense_invert(int64_t ld, double *M, double *D, int32_t *fail, hipStream_t st, int64_t n, double *P,
                         int32_t *rowperm, int32_t *stats, double u) {
    const int64_t nb = ld / DB;
    for (int64_t k = 0; k < nb; ++k) {
        if (u > 0.0 && P) {  // (P: n x 64 for the panel, then PANEL_FAST for the fast path)
            double *S = P + n * DB;
            const int64_t rows = n - k * DB - DB;  // below the tile
            k_panel_tile<false><<<1, DTPB, 0, st>>>(nullptr, n, ld, (int)k, M, S);
            if (rows > 0)
                k_panel_rows<false><<<dim3((unsigned)((rows + PRTPB - 1) / PRTPB), 1), PRTPB, 0, st>>>(nullptr, n, ld,
                                                                                                     (int)k, M, S);
            k_dense_panel_pivot<<<1, DTPB, 0, st>>>(n, ld, k, M, P, rowperm, stats, u, S);
        }
        k_gj_diag<<<1, DTPB, 0, st>>>(ld, k, M, D, fail);
        k_gj_rowpanel<<<(unsigned)nb, DTPB, 0, st>>>(ld, k, D, M);
        if (nb > 1) {
            k_gj_update<<<dim3((unsigned)(nb - 1), (unsigned)(nb - 1)), DTPB, 0, st>>>(ld, k, M);
            k_gj_colpanel<<<(unsigned)(nb - 1), DTPB, 0, st>>>(ld, k, D, M);
        }
    }
}

// y = alpha * M x + beta * y over the leading n x n block: one wave per row,
// 16-byte loads of the row (ld is a multiple of 64 doubles), x from L2.
typedef double dn_d2 __attribute__((ext_vector_type(2)));
// (xp: x permuted, xp[c] = x[rowperm[c]] -- the threshold-pivoted inverse is (Pi M)^-1)
__global__ __launch_bounds__(256) void k_dense_gemv(int64_t n, int64_t ld, const double *__restrict__ M,
                                                    const double *__restrict__ x, double *__restrict__ y,
                                                    const int32_t *__restrict__ rowperm) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const int lane = threadIdx.x & 63;
    const double *row = M + i * ld;
    double acc = 0.0;
    const int64_t n2 = n & ~(int64_t)1;
    auto xa = [&](int64_t c) { return rowperm ? x[rowperm[c]] : x[c]; };
    for (int64_t c = 2 * lane; c < n2; c += 128) {
        const dn_d2 m = __builtin_nontemporal_load(reinterpret_cast<const dn_d2 *>(row + c));
        acc += m.x * xa(c);
        acc += m.y * xa(c + 1);
    }
    if ((n & 1) && lane == 0) acc += row[n - 1] * xa(n - 1);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) y[i] = acc;
}
void launch_dense_gemv(int64_t n, int64_t ld, const double *M, const double *x, double *y, hipStream_t st,
                       const int32_t *rowperm) {
    if (n > 0) k_dense_gemv<<<(unsigned)((n + 3) / 4), 256, 0, st>>>(n, ld, M, x, y, rowperm);
}

// Block-diagonal GEMV: one wave per row, the row of its chunk's block.
__global__ __launch_bounds__(256) void k_bdense_gemv(int64_t n, int64_t ld, const int32_t *__restrict__ cof,
                                                     const int64_t *__restrict__ cptr, const double *__restrict__ M,
                                                     const double *__restrict__ x, double *__restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const int lane = threadIdx.x & 63;
    const int64_t c = cof[i], c0 = cptr[c], len = cptr[c + 1] - c0;
    const double *row = M + c * ld * ld + (i - c0) * ld;
    const double *xc = x + c0;
    double acc = 0.0;
    const int64_t n2 = len & ~(int64_t)1;
    for (int64_t k = 2 * lane; k < n2; k += 128) {
        const dn_d2 m = __builtin_nontemporal_load(reinterpret_cast<const dn_d2 *>(row + k));
        acc += m.x * xc[k];
        acc += m.y * xc[k + 1];
    }
    if ((len & 1) && lane == 0) acc += row[len - 1] * xc[len - 1];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) y[i] = acc;
}
void launch_bdense_gemv(int64_t n, int64_t ld, const int32_t *cof, const int64_t *cptr, const double *M,
                        const double *x, double *y, hipStream_t st) {
    if (n > 0) k_bdense_gemv<<<(unsigned)((n + 3) / 4), 256, 0, st>>>(n, ld, cof, cptr, M, x, y);
}

__global__ __launch_bounds__(256) void k_dense_rowscale(int64_t n, int64_t ld, const double *d, double *M) {
    const int64_t r = blockIdx.y;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r < n && j < ld) M[r * ld + j] = M[r * ld + j] * d[r];
}
void launch_dense_rowscale(int64_t n, int64_t ld, const double *d, double *M, hipStream_t st) {
    if (n > 0) k_dense_rowscale<<<dim3((unsigned)((ld + 255) / 256), (unsigned)n), 256, 0, st>>>(n, ld, d, M);
}

// C = A B on 64 x 64 tiles (blockIdx = (tile column, tile row)), 4 x 4 outputs per thread
__global__ __launch_bounds__(DTPB) void k_dense_gemm(int64_t ld, const double *A, const double *B, double *C) {
    __shared__ double at[DB][DB + 1];  // A_ik^T
    __shared__ double b[DB][DB + 1];   // B_kj
    const int64_t j = blockIdx.x, i = blockIdx.y, nb = ld / DB;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    double acc[4][4] = {};
    for (int64_t k = 0; k < nb; ++k) {
        __syncthreads();
        tile_load(A + (i * DB) * ld + k * DB, ld, at, true);
        tile_load(B + (k * DB) * ld + j * DB, ld, b, false);
        __syncthreads();
        for (int kk = 0; kk < DB; ++kk) {
            double av[4], bv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) av[r] = at[kk][ty + 16 * r];
#pragma unroll
            for (int q = 0; q < 4; ++q) bv[q] = b[kk][tx + 16 * q];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[r][q] += av[r] * bv[q];
        }
    }
    double *Ct = C + (i * DB) * ld + j * DB;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) Ct[(int64_t)(ty + 16 * r) * ld + tx + 16 * q] = acc[r][q];
}
void launch_dense_gemm(int64_t ld, const double *A, const double *B, double *C, hipStream_t st) {
    const unsigned nb = (unsigned)(ld / DB);
    if (nb) k_dense_gemm<<<dim3(nb, nb), DTPB, 0, st>>>(ld, A, B, C);
}

// ============================================ multifrontal LU (sparse_lu.cpp) ==
// A front's tile (I, J) (64 x 64, leading dimension ld = 64 ldt).
__device__ __forceinline__ double *mf_tile(const MFront &f, double *W, int64_t I, int64_t J) {
    const int64_t ld = (int64_t)f.ldt * DB;
    return W + f.ws + (I * DB) * ld + J * DB;
}

__global__ __launch_bounds__(256) void k_mf_pad(const MFront *F, double *W) {
    const MFront f = F[blockIdx.y];
    const int64_t r = f.p + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r < (int64_t)f.pt * DB) W[f.ws + r * ((int64_t)f.ldt * DB) + r] = 1.0;
}
void launch_mf_pad(int nf, const MFront *F, int max_pad, double *W, hipStream_t st) {
    if (nf > 0 && max_pad > 0) k_mf_pad<<<dim3((unsigned)((max_pad + 255) / 256), (unsigned)nf), 256, 0, st>>>(F, W);
}

__global__ __launch_bounds__(256) void k_mf_scatter(int64_t m, const int64_t *dst, const int64_t *src,
                                                    const double *val, double *W) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k < m) W[dst[k]] = val[src[k]];
}
void launch_mf_scatter(int64_t m, const int64_t *dst, const int64_t *src, const double *val, double *W,
                       hipStream_t st) {
    if (m > 0) k_mf_scatter<<<(unsigned)((m + 255) / 256), 256, 0, st>>>(m, dst, src, val, W);
}

// blockIdx.x: child, blockIdx.y: update row of the child
__global__ __launch_bounds__(256) void k_mf_extend(const MChild *C, const int32_t *maps, const double *Wprev,
                                                   double *Wcur) {
    const MChild c = C[blockIdx.x];
    const int64_t r = blockIdx.y;
    if (r >= c.q) return;
    const int64_t pr = maps[c.map_off + r];
    const double *src = Wprev + c.src_ws + ((int64_t)c.src_pp + r) * c.src_ld + c.src_pp;
    double *dst = Wcur + c.dst_ws + pr * c.dst_ld;
    for (int64_t s = threadIdx.x; s < c.q; s += 256) {
        const int64_t ps = maps[c.map_off + s];
        dst[ps] = dst[ps] + src[s];
    }
}
void launch_mf_extend(int nc, const MChild *C, int max_q, const int32_t *maps, const double *Wprev, double *Wcur,
                      hipStream_t st) {
    if (nc > 0 && max_q > 0) k_mf_extend<<<dim3((unsigned)nc, (unsigned)max_q), 256, 0, st>>>(C, maps, Wprev, Wcur);
}

// Gauss-Jordan step k, as launch_dense_invert but over the front's pivot tiles
// only and batched over fronts (blockIdx.z).  The block elimination only needs
// D = T_kk^-1, however it is computed; saddle-point blocks (the 2-way fp block:
// zero pressure diagonal) have zero scalar pivots whose tile is still regular.
// D is formed as LAPACK's getrf + getrs on the identity: LU with partial
// pivoting in LDS, then L^-1 and U^-1 applied to P I.  (Round 3 formed it by
// scalar Gauss-Jordan with partial pivoting: on footing's undrained solid
// block -- Dirichlet rows of unit diagonal next to entries of 1e6 -- that left
// ||K y - x|| / ||x|| at 2.4e-6 .. 7.9e-6 with 64-row leaves, where the LU
// inverse gives 7.9e-11, LAPACK's own level; CPU restatement in
// tools/mf_emulate.py.)
#pragma clang fp contract(off)
// fail[0]: a zero pivot with static pivoting off (tau = 0); fail[1]: pivots replaced by +-tau
__global__ __launch_bounds__(DTPB) void k_mf_gj_diag(const MFront *F, int k, double *W, double *D, int32_t *fail,
                                                     double tau) {
    __shared__ double a[DB][DB + 1];
    __shared__ double v[DB][DB + 1];
    __shared__ int prow;
    const MFront f = F[blockIdx.z];
    if (k >= f.pt) return;
    const int64_t ld = (int64_t)f.ldt * DB;
    const double *src = mf_tile(f, W, k, k);
    for (int t = threadIdx.x; t < DB * DB; t += DTPB) {
        const int i = t / DB, j = t % DB;
        a[i][j] = src[(int64_t)i * ld + j];
        v[i][j] = i == j ? 1.0 : 0.0;
    }
    __syncthreads();
    // LU with partial pivoting: a := L \ U (unit L below the diagonal), rows of v = P I swapped alike
    for (int p = 0; p < DB; ++p) {
        if (threadIdx.x < DB) {  // wave 0: argmax |a[i][p]|, i >= p (ties: the smaller row)
            const int i = threadIdx.x;
            double m = i >= p ? fabs(a[i][p]) : -1.0;
            int r = i;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const double m2 = __shfl_xor(m, o);
                const int r2 = __shfl_xor(r, o);
                if (m2 > m || (m2 == m && r2 < r)) {
                    m = m2;
                    r = r2;
                }
            }
            if (i == 0) prow = r;
        }
        __syncthreads();
        const int r = prow;
        if (r != p && threadIdx.x < 2 * DB) {  // swap rows p and r of [a | v]
            const int j = threadIdx.x & (DB - 1);
            double (*m)[DB + 1] = threadIdx.x < DB ? a : v;
            const double t = m[p][j];
            m[p][j] = m[r][j];
            m[r][j] = t;
        }
        __syncthreads();
        double piv = a[p][p];
        __syncthreads();  // every wave holds the pivot before a[p][p] may change
        if (fabs(piv) <= tau && k * DB + p < f.p) {  // static pivot (MUMPS CNTL(4) semantics), not on the padding
            if (tau <= 0.0) {
                if (threadIdx.x == 0) atomicOr(fail, 1);
                return;  // uniform across the workgroup: every thread read the same pivot
            }
            piv = piv < 0.0 ? -tau : tau;
            if (threadIdx.x == 0) {
                a[p][p] = piv;
                atomicAdd(fail + 1, 1);
            }
        }
        if (threadIdx.x > p && threadIdx.x < DB) a[threadIdx.x][p] = a[threadIdx.x][p] / piv;  // l_ip
        __syncthreads();
        for (int t = threadIdx.x; t < DB * DB; t += DTPB) {  // trailing update
            const int i = t / DB, j = t % DB;
            if (i > p && j > p) a[i][j] = a[i][j] - a[i][p] * a[p][j];
        }
        __syncthreads();
    }
    // v := L^-1 v
    for (int p = 0; p < DB - 1; ++p) {
        for (int t = threadIdx.x; t < DB * DB; t += DTPB) {
            const int i = t / DB, j = t % DB;
            if (i > p) v[i][j] = v[i][j] - a[i][p] * v[p][j];
        }
        __syncthreads();
    }
    // v := U^-1 v
    for (int p = DB - 1; p >= 0; --p) {
        if (threadIdx.x < DB) v[p][threadIdx.x] = v[p][threadIdx.x] / a[p][p];
        __syncthreads();
        for (int t = threadIdx.x; t < p * DB; t += DTPB) {
            const int i = t / DB, j = t % DB;
            v[i][j] = v[i][j] - a[i][p] * v[p][j];
        }
        __syncthreads();
    }
    double *Dt = D + (int64_t)blockIdx.z * DB * DB;
    for (int t = threadIdx.x; t < DB * DB; t += DTPB) Dt[t] = v[t / DB][t % DB];
}
#pragma clang fp contract(on)

__device__ __forceinline__ void mf_mm(const double *A, int64_t lda, const double *B, int64_t ldb,
                                      double (*at)[DB + 1], double (*b)[DB + 1], double acc[4][4]) {
    tile_load(A, lda, at, true);
    tile_load(B, ldb, b, false);
    __syncthreads();
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    for (int kk = 0; kk < DB; ++kk) {
        double av[4], bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) av[r] = at[kk][ty + 16 * r];
#pragma unroll
        for (int q = 0; q < 4; ++q) bv[q] = b[kk][tx + 16 * q];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] += av[r] * bv[q];
    }
}

// row panel: F_kj := D F_kj (j != k), F_kk := D
__global__ __launch_bounds__(DTPB) void k_mf_gj_rowpanel(const MFront *F, int k, double *W, const double *D) {
    __shared__ double at[DB][DB + 1];
    __shared__ double b[DB][DB + 1];
    const MFront f = F[blockIdx.z];
    const int64_t j = blockIdx.x;
    if (k >= f.pt || j >= f.ldt) return;
    const int64_t ld = (int64_t)f.ldt * DB;
    const double *Dt = D + (int64_t)blockIdx.z * DB * DB;
    double *C = mf_tile(f, W, k, j);
    if (j == k) {
        for (int t = threadIdx.x; t < DB * DB; t += DTPB) C[(int64_t)(t / DB) * ld + t % DB] = Dt[t];
        return;
    }
    double acc[4][4] = {};
    mf_mm(Dt, DB, C, ld, at, b, acc);
    __syncthreads();
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) C[(int64_t)(ty + 16 * r) * ld + tx + 16 * q] = acc[r][q];
}

// update: F_ij -= F_ik F_kj (i, j != k)
__global__ __launch_bounds__(DTPB) void k_mf_gj_update(const MFront *F, int k, double *W) {
    __shared__ double at[DB][DB + 1];
    __shared__ double b[DB][DB + 1];
    const MFront f = F[blockIdx.z];
    if (k >= f.pt || (int)blockIdx.x >= f.ldt - 1 || (int)blockIdx.y >= f.ldt - 1) return;
    const int64_t j = blockIdx.x + (blockIdx.x >= (unsigned)k ? 1 : 0);
    const int64_t i = blockIdx.y + (blockIdx.y >= (unsigned)k ? 1 : 0);
    const int64_t ld = (int64_t)f.ldt * DB;
    double acc[4][4] = {};
    mf_mm(mf_tile(f, W, i, k), ld, mf_tile(f, W, k, j), ld, at, b, acc);
    double *C = mf_tile(f, W, i, j);
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double *c = C + (int64_t)(ty + 16 * r) * ld + tx + 16 * q;
            *c = *c - acc[r][q];
        }
}

// column panel: F_ik := -F_ik D (i != k)
__global__ __launch_bounds__(DTPB) void k_mf_gj_colpanel(const MFront *F, int k, double *W, const double *D) {
    __shared__ double at[DB][DB + 1];
    __shared__ double b[DB][DB + 1];
    const MFront f = F[blockIdx.z];
    if (k >= f.pt || (int)blockIdx.x >= f.ldt - 1) return;
    const int64_t i = blockIdx.x + (blockIdx.x >= (unsigned)k ? 1 : 0);
    const int64_t ld = (int64_t)f.ldt * DB;
    double *C = mf_tile(f, W, i, k);
    double acc[4][4] = {};
    mf_mm(C, ld, D + (int64_t)blockIdx.z * DB * DB, DB, at, b, acc);
    __syncthreads();
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) C[(int64_t)(ty + 16 * r) * ld + tx + 16 * q] = -acc[r][q];
}

void launch_mf_panel_pivot(int nf, const MFront *F, const int64_t *pst, const int64_t *soff, int k, double *W,
                           double *P, int32_t *rowperm, int32_t *stats, double u, hipStream_t st, int32_t *dflag,
                           double *S, int64_t max_rows) {
    if (nf <= 0 || u <= 0.0) return;
    if (S) {
        k_panel_tile<true><<<(unsigned)nf, DTPB, 0, st>>>(F, 0, 0, k, W, S);
        const int64_t rows = max_rows - (int64_t)k * DB;  // (bound on every front's panel rows at step k)
        if (rows > 0)
            k_panel_rows<true><<<dim3((unsigned)((rows + PRTPB - 1) / PRTPB), (unsigned)nf), PRTPB, 0, st>>>(F, 0, 0, k,
                                                                                                           W, S);
    }
    k_mf_panel_pivot<<<(unsigned)nf, DTPB, 0, st>>>(F, pst, soff, k, W, P, rowperm, stats, u, dflag, S);
}
int panel_fast_doubles() { return PANEL_FAST; }
void launch_mf_gj_step(int nf, const MFront *F, int max_ldt, int k, double *W, double *D, int32_t *fail,
                       double tau, hipStream_t st) {
    if (nf <= 0 || max_ldt <= 0) return;
    k_mf_gj_diag<<<dim3(1, 1, (unsigned)nf), DTPB, 0, st>>>(F, k, W, D, fail, tau);
    k_mf_gj_rowpanel<<<dim3((unsigned)max_ldt, 1, (unsigned)nf), DTPB, 0, st>>>(F, k, W, D);
    if (max_ldt > 1) {
        k_mf_gj_update<<<dim3((unsigned)(max_ldt - 1), (unsigned)(max_ldt - 1), (unsigned)nf), DTPB, 0, st>>>(F, k, W);
        k_mf_gj_colpanel<<<dim3((unsigned)(max_ldt - 1), 1, (unsigned)nf), DTPB, 0, st>>>(F, k, W, D);
    }
}

// blockIdx.x: front row (U part rows [0, p), then X part rows from pp), blockIdx.y: front.
// Compact layout (no tile padding): U row r = [F11^-1 | F11^-1 F12] (p + q), X row = p.
__global__ __launch_bounds__(256) void k_mf_store(const MFront *F, const MStore *S, const double *W, double *U,
                                                  double *X) {
    const MFront f = F[blockIdx.y];
    const MStore s = S[blockIdx.y];
    const int64_t r = blockIdx.x, ld = (int64_t)f.ldt * DB, pp = (int64_t)f.pt * DB, p = f.p, q = f.q;
    const double *src = W + f.ws + r * ld;
    if (r < p) {
        double *dst = U + s.uoff + r * (p + q);
        for (int64_t c = threadIdx.x; c < p + q; c += 256) dst[c] = src[c < p ? c : pp + (c - p)];
    } else if (r >= pp && r < pp + q) {
        double *dst = X + s.xoff + (r - pp) * p;
        for (int64_t c = threadIdx.x; c < p; c += 256) dst[c] = src[c];
    }
}
void launch_mf_store(int nf, const MFront *F, const MStore *S, int max_rows, const double *W, double *U, double *X,
                     hipStream_t st) {
    if (nf > 0 && max_rows > 0) k_mf_store<<<dim3((unsigned)max_rows, (unsigned)nf), 256, 0, st>>>(F, S, W, U, X);
}

// ---------------------------------------------------------------- solve --
__global__ __launch_bounds__(256) void k_mf_fwd_gather(int64_t m, const int32_t *rf, const int32_t *rl,
                                                       const MSolve *S, const int64_t *cptr, const int64_t *cidx,
                                                       const double *b, const double *cu, double *z, double *acc) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= m) return;
    const MSolve s = S[rf[k]];
    const int64_t r = rl[k];
    double v = r < s.p ? b[s.pstart + r] : 0.0;
    for (int64_t t = cptr[k]; t < cptr[k + 1]; ++t) v += cu[cidx[t]];
    if (r < s.p) z[s.pstart + r] = v;
    else acc[s.qoff + r - s.p] = v;
}
void launch_mf_fwd_gather(int64_t m, const int32_t *rf, const int32_t *rl, const MSolve *S, const int64_t *cptr,
                          const int64_t *cidx, const double *b, const double *cu, double *z, double *acc,
                          hipStream_t st) {
    if (m > 0) k_mf_fwd_gather<<<(unsigned)((m + 255) / 256), 256, 0, st>>>(m, rf, rl, S, cptr, cidx, b, cu, z, acc);
}

__global__ __launch_bounds__(256) void k_mf_fwd_gemv(int64_t m, const int32_t *rf, const int32_t *rl,
                                                     const MSolve *S, const double *__restrict__ X,
                                                     const double *__restrict__ z, const double *acc, double *cu) {
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= m) return;
    const int lane = threadIdx.x & 63;
    const MSolve s = S[rf[k]];
    const int64_t i = rl[k];
    const double *row = X + s.xoff + i * s.pp;
    const double *zp = z + s.pstart;
    double a = 0.0;
    for (int64_t j = lane; j < s.p; j += 64) a += row[j] * zp[j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
    if (lane == 0) cu[s.qoff + i] = acc[s.qoff + i] + a;
}
void launch_mf_fwd_gemv(int64_t m, const int32_t *rf, const int32_t *rl, const MSolve *S, const double *X,
                        const double *z, const double *acc, double *cu, hipStream_t st) {
    if (m > 0) k_mf_fwd_gemv<<<(unsigned)((m + 3) / 4), 256, 0, st>>>(m, rf, rl, S, X, z, acc, cu);
}

__global__ __launch_bounds__(256) void k_mf_bwd(int64_t m, const int32_t *rf, const int32_t *rl, const MSolve *S,
                                                const double *__restrict__ U, const int32_t *__restrict__ slist,
                                                const double *__restrict__ z, double *x) {
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= m) return;
    const int lane = threadIdx.x & 63;
    const MSolve s = S[rf[k]];
    const int64_t r = rl[k];
    const double *row = U + s.uoff + r * s.ld;
    const double *zp = z + s.pstart;
    double a = 0.0;
    for (int64_t j = lane; j < s.p; j += 64) a += row[j] * zp[j];
    const double *g = row + s.pp;
    const int32_t *sl = slist + s.soff;
    for (int64_t j = lane; j < s.q; j += 64) a -= g[j] * x[sl[j]];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
    if (lane == 0) x[s.pstart + r] = a;
}
void launch_mf_bwd(int64_t m, const int32_t *rf, const int32_t *rl, const MSolve *S, const double *U,
                   const int32_t *slist, const double *z, double *x, hipStream_t st) {
    if (m > 0) k_mf_bwd<<<(unsigned)((m + 3) / 4), 256, 0, st>>>(m, rf, rl, S, U, slist, z, x);
}

__global__ __launch_bounds__(256) void k_gather_i32(int64_t n, const int32_t *perm, const double *b, double *x) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) x[i] = b[perm[i]];
}
__global__ __launch_bounds__(256) void k_scatter_i32(int64_t n, const int32_t *perm, const double *x, double *y) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[perm[i]] = x[i];
}
void launch_gather_i32(int64_t n, const int32_t *perm, const double *b, double *x, hipStream_t st) {
    if (n > 0) k_gather_i32<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, perm, b, x);
}
void launch_scatter_i32(int64_t n, const int32_t *perm, const double *x, double *y, hipStream_t st) {
    if (n > 0) k_scatter_i32<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, perm, x, y);
}

}  // namespace pls
