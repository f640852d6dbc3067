// kernels.hip -- HIP kernels for gfx950 (MI355X / CDNA4) behind libpls.so.
//
// Everything on the solver path is HBM-bandwidth bound fp64 sparse / BLAS-1
// work (no MFMA).  Design rules applied (cdna_hip_programming.md):
//  * 64-lane wavefronts: CSR rows are mapped to groups of LPR lanes
//    (LPR in {8,16,32,64}) sized from the mean row length, reductions are
//    __shfl_xor trees inside the group;
//  * val / col streams use non-temporal loads (read once), the x gathers go
//    through L2 / the Infinity Cache (banded columns: hot window);
//  * reductions are deterministic: a fixed grid that depends only on n, one
//    partial per block, then a single-block final pass in fixed order, so a
//    solve is bitwise reproducible run to run;
//  * the ILU(0) factor and sweeps are level scheduled; the triangular factors
//    are stored in level order so each level streams a contiguous slice.
#include "kernels.hpp"

#include <hipcub/hipcub.hpp>

#include <cstdio>

namespace pls {

static constexpr int TPB = 256;

static inline unsigned grid_for(int64_t work, int per_block) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    return (unsigned)g;
}


__device__ __forceinline__ double wave_reduce(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}


// Partial dot of a CSR row slice over LPR lanes, U entries per lane in flight:
// unconditional loads at a clamped index (s is valid inside the loop) and a
// masked value, so the loads of one pass issue back to back.
template <int LPR, int U, bool NT>
__device__ __forceinline__ double row_dot(int64_t s, int64_t e, int sub, const int32_t *__restrict__ ci,
                                          const double *__restrict__ val, const double *x) {
    double acc = 0.0;
    for (int64_t k0 = s; k0 < e; k0 += U * LPR) {
        int32_t c[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t k = k0 + u * LPR + sub;
            const int64_t kk = k < e ? k : s;
            if (NT) {
                c[u] = __builtin_nontemporal_load(ci + kk);
                const double t = __builtin_nontemporal_load(val + kk);
                v[u] = k < e ? t : 0.0;
            } else {
                c[u] = ci[kk];
                const double t = val[kk];
                v[u] = k < e ? t : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u] * x[(uint32_t)c[u]];
    }
    return acc;
}

// ============================================================ synthetic ====
// Bit-exact restatement of the synthetic spec; every float
// expression rounds as written (no FMA contraction) so the device matrices are
// identical to the CPU definition.
#pragma clang fp contract(off)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t hash3(uint64_t s, uint64_t a, uint64_t b) {
    return mix64(mix64(mix64(s) ^ a) ^ b);
}
__device__ __forceinline__ double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }

#define SALT_VAL 0x5A1BE5ULL
#define SALT_DIAGA 0xD1A60AULL
#define SALT_DIAGP 0xD1A60BULL
#define SALT_BC 0x00BC00ULL
#define SALT_RHS 0x00B0B0ULL

__device__ __forceinline__ int blk_id(int a, int b) {
    // ss sf sp / sf ff fp / sp fp pp
    const int t = a * 3 + b;
    return (t == 0) ? 0 : (t == 1 || t == 3) ? 1 : (t == 2 || t == 6) ? 2 : (t == 4) ? 3 : (t == 5 || t == 7) ? 4 : 5;
}

__device__ __forceinline__ int field_of(const SynthDev &S, int64_t g) {
    return g < S.off[1] ? 0 : (g < S.off[2] ? 1 : 2);
}

// Visits the global columns of row i (local in field a) in ascending order.
template <typename F>
__device__ __forceinline__ void synth_visit(const SynthDev &S, int a, int64_t i, F &&f) {
    for (int b = 0; b < 3; ++b) {
        const int bid = blk_id(a, b);
        const int32_t *D = S.offs[bid];
        const int m = S.cnt[bid];
        const int64_t na = S.n[a], nb = S.n[b];
        if (a <= b) {
            const int64_t ctr = (a == b) ? i : (i * nb) / na;
            for (int k = 0; k < m; ++k) {
                const int64_t j = ctr + D[k];
                if (j >= 0 && j < nb) f(b, S.off[b] + j);
            }
        } else {
            for (int k = m - 1; k >= 0; --k) {
                const int64_t mm = i - D[k];
                if (mm < 0 || mm >= na) continue;
                const int64_t lo = (mm * nb + na - 1) / na;
                int64_t hi = ((mm + 1) * nb + na - 1) / na;
                if (hi > nb) hi = nb;
                for (int64_t j = lo; j < hi; ++j) f(b, S.off[b] + j);
            }
        }
    }
}

__device__ __forceinline__ int64_t synth_global_row(const SynthDev &S, int64_t l) {
    const int f = l < S.rloff[1] ? 0 : (l < S.rloff[2] ? 1 : 2);
    return S.off[f] + S.rlo[f] + (l - S.rloff[f]);
}

__global__ __launch_bounds__(TPB) void k_synth_count(SynthDev S, int64_t *row_len) {
    const int64_t n = S.nrows;
    const int64_t l = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (l > n) return;
    if (l == n) { row_len[n] = 0; return; }
    const int64_t g = synth_global_row(S, l);
    const int a = field_of(S, g);
    int64_t c = 0;
    synth_visit(S, a, g - S.off[a], [&](int, int64_t) { ++c; });
    row_len[l] = c;
}

__global__ __launch_bounds__(TPB) void k_synth_fill(SynthDev S, int variant, const int64_t *rp,
                                                    int32_t *col, double *val) {
    const int64_t l = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (l >= S.nrows) return;
    const int64_t g = synth_global_row(S, l);
    const int a = field_of(S, g);
    const int64_t i = g - S.off[a];
    const uint64_t sv = S.seed ^ SALT_VAL;
    const uint64_t sd = S.seed ^ (variant == 0 ? SALT_DIAGA : SALT_DIAGP);
    const bool bcrow = (variant == 2 && a == 2 &&
                        ((hash3(S.seed ^ SALT_BC, (uint64_t)i, 7ULL) & 15ULL) == 0ULL));
    int64_t pos = rp[l];
    int64_t dpos = -1;
    double sum = 0.0;
    synth_visit(S, a, i, [&](int b, int64_t gj) {
        col[pos] = (int32_t)gj;
        if (gj == g) {
            dpos = pos;
            val[pos] = 0.0;
        } else {
            const uint64_t lo = (uint64_t)(g < gj ? g : gj), hi = (uint64_t)(g < gj ? gj : g);
            const double u = u01(hash3(sv, lo, hi));
            const double v = (a == b) ? -u : -(0.1 * u);
            val[pos] = bcrow ? 0.0 : v;
            sum = sum + fabs(v);
        }
        ++pos;
    });
    if (dpos >= 0) {
        if (bcrow) {
            val[dpos] = 1.0;
        } else {
            const double u = u01(hash3(sd, (uint64_t)g, (uint64_t)g));
            const double sh = S.delta * (1.0 + u);
            val[dpos] = sum + sh;
        }
    }
}

__global__ __launch_bounds__(TPB) void k_synth_rhs(SynthDev S, uint64_t seed, double *b) {
    const int64_t l = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (l >= S.nrows) return;
    const int64_t i = synth_global_row(S, l);
    const double u = u01(hash3(seed ^ SALT_RHS, (uint64_t)i, 3ULL));
    b[l] = 2.0 * u - 1.0;
}

#pragma clang fp contract(on)

void launch_synth_count(const SynthDev &S, int64_t *row_len, hipStream_t st) {
    k_synth_count<<<grid_for(S.nrows + 1, TPB), TPB, 0, st>>>(S, row_len);
}
void launch_synth_fill(const SynthDev &S, int variant, const int64_t *row_ptr, int32_t *col,
                       double *val, hipStream_t st) {
    if (S.nrows > 0) k_synth_fill<<<grid_for(S.nrows, TPB), TPB, 0, st>>>(S, variant, row_ptr, col, val);
}
void launch_synth_rhs(const SynthDev &S, uint64_t seed, double *b, hipStream_t st) {
    if (S.nrows > 0) k_synth_rhs<<<grid_for(S.nrows, TPB), TPB, 0, st>>>(S, seed, b);
}

// ================================================================ scans ====
size_t exclusive_scan_tmp_bytes(int64_t n) {
    size_t bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int64_t *)nullptr, (int64_t *)nullptr,
                                     (int)(n + 1));
    return bytes;
}
void exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n, void *tmp, size_t tmp_bytes,
                        hipStream_t st) {
    (void)hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, (int)(n + 1), st);
}

// ========================================================== extraction =====
// Block of a row: explicit starts (binary search; nb + 1 entries) or PETSc's
// sizes (n / nb, the first n % nb blocks one longer).  b0 / len of the block.
__device__ __forceinline__ int64_t block_of(int64_t i, int64_t n, int64_t nb, const int64_t *bstart, int64_t &b0,
                                            int64_t &len) {
    if (bstart) {
        int64_t lo = 0, hi = nb;  // largest b with bstart[b] <= i
        while (hi - lo > 1) {
            const int64_t m = (lo + hi) >> 1;
            if (bstart[m] <= i) lo = m; else hi = m;
        }
        b0 = bstart[lo];
        len = bstart[lo + 1] - b0;
        return lo;
    }
    const int64_t q = n / nb, r = n % nb;
    const int64_t b = i < r * (q + 1) ? i / (q + 1) : r + (i - r * (q + 1)) / q;
    b0 = b * q + (b < r ? b : r);
    len = q + (b < r ? 1 : 0);
    return b;
}
__device__ __forceinline__ void block_range(int64_t b, int64_t n, int64_t nb, const int64_t *bstart, int64_t &b0,
                                            int64_t &len) {
    if (bstart) {
        b0 = bstart[b];
        len = bstart[b + 1] - b0;
        return;
    }
    const int64_t q = n / nb, r = n % nb;
    b0 = b * q + (b < r ? b : r);
    len = q + (b < r ? 1 : 0);
}

__device__ __forceinline__ void window_of(const WindowSpec &w, int64_t lr, int64_t nloc, int64_t r0,
                                          int64_t &lo, int64_t &hi) {
    if (w.mode == 0) {
        lo = w.c0;
        hi = w.c1;
        return;
    }
    int64_t b0, len;
    block_of(lr, nloc, w.nblocks, w.bstart, b0, len);
    lo = r0 + b0;
    hi = r0 + b0 + len;
}

__device__ __forceinline__ int64_t lower_bound_i32(const int32_t *a, int64_t s, int64_t e, int64_t v) {
    while (s < e) {
        const int64_t m = (s + e) >> 1;
        if ((int64_t)a[m] < v) s = m + 1; else e = m;
    }
    return s;
}

__global__ __launch_bounds__(TPB) void k_extract_count(const int64_t *rp, const int32_t *ci, int64_t r0,
                                                       int64_t r1, WindowSpec w, int64_t *len) {
    const int64_t nloc = r1 - r0;
    const int64_t lr = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (lr > nloc) return;
    if (lr == nloc) { len[nloc] = 0; return; }
    const int64_t r = r0 + lr;
    int64_t lo, hi;
    window_of(w, lr, nloc, r0, lo, hi);
    const int64_t a = lower_bound_i32(ci, rp[r], rp[r + 1], lo);
    const int64_t b = lower_bound_i32(ci, a, rp[r + 1], hi);
    len[lr] = b - a;
}

__global__ __launch_bounds__(TPB) void k_extract_fill(const int64_t *rp, const int32_t *ci, const double *val,
                                                      int64_t r0, int64_t r1, WindowSpec w, int64_t cshift,
                                                      const int64_t *orp, int32_t *oci, double *oval) {
    const int64_t nloc = r1 - r0;
    // one wave per row: contiguous copy
    const int64_t lr = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (lr >= nloc) return;
    const int64_t r = r0 + lr;
    int64_t lo, hi;
    window_of(w, lr, nloc, r0, lo, hi);
    const int64_t a = lower_bound_i32(ci, rp[r], rp[r + 1], lo);
    const int64_t dst = orp[lr];
    const int64_t cnt = orp[lr + 1] - dst;
    for (int64_t k = lane; k < cnt; k += 64) {
        oci[dst + k] = (int32_t)((int64_t)ci[a + k] - cshift);
        oval[dst + k] = val[a + k];
    }
}

void launch_extract_count(const int64_t *rp, const int32_t *ci, int64_t r0, int64_t r1, WindowSpec w,
                          int64_t *row_len, hipStream_t st) {
    k_extract_count<<<grid_for(r1 - r0 + 1, TPB), TPB, 0, st>>>(rp, ci, r0, r1, w, row_len);
}
void launch_extract_fill(const int64_t *rp, const int32_t *ci, const double *val, int64_t r0, int64_t r1,
                         WindowSpec w, int64_t cshift, const int64_t *out_rp, int32_t *out_ci,
                         double *out_val, hipStream_t st) {
    k_extract_fill<<<grid_for((r1 - r0) * 64, TPB), TPB, 0, st>>>(rp, ci, val, r0, r1, w, cshift, out_rp,
                                                                  out_ci, out_val);
}

// ================================================================= SpMV ====
// y = alpha * (M x) + beta * z.  LPR lanes per row; 256 / LPR rows per block.
template <int LPR>
__global__ __launch_bounds__(TPB) void k_spmv(int64_t nrows, const int64_t *__restrict__ rp,
                                              const int32_t *__restrict__ ci, const double *__restrict__ val,
                                              const double *__restrict__ x, double *__restrict__ y,
                                              double alpha, double beta, const double *__restrict__ z) {
    const int sub = threadIdx.x & (LPR - 1);
    const int64_t row = ((int64_t)blockIdx.x * TPB + threadIdx.x) / LPR;
    if (row >= nrows) return;
    const int64_t s = rp[row], e = rp[row + 1];
    double acc = row_dot<LPR, 4, true>(s, e, sub, ci, val, x);
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (sub == 0) {
        double r = alpha * acc;
        if (beta != 0.0) r += beta * z[row];
        y[row] = r;
    }
}

// Short rows (mean < 12 nnz: AMG interpolation P, ~7 per row), opt-in
// (pls.spmv_short 1): one lane per row, entries in CSR order (scipy's per-row
// order), eight loads of each kind issued before the x gathers.  Measured
// slower than 8 lanes per row (k_spmv<8>) on the N=59 level-0 prolongation
// P e (561-596 vs ~400 us): a load instruction touches 64 rows' k-th entries,
// ~84 cache lines, and the texture path issues them a few lanes per cycle.
__global__ __launch_bounds__(TPB) void k_spmv_short(int64_t nrows, const int64_t *__restrict__ rp,
                                                    const int32_t *__restrict__ ci, const double *__restrict__ val,
                                                    const double *__restrict__ x, double *__restrict__ y,
                                                    double alpha, double beta, const double *__restrict__ z) {
    const int64_t row = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (row >= nrows) return;
    const int64_t s = rp[row], e = rp[row + 1];
    const double zr = beta != 0.0 ? z[row] : 0.0;
    double acc = 0.0;
    for (int64_t k0 = s; k0 < e; k0 += 8) {
        int32_t c[8];
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t k = k0 + u < e ? k0 + u : s;  // (clamped: the value is zeroed)
            c[u] = __builtin_nontemporal_load(ci + k);
            const double vv = __builtin_nontemporal_load(val + k);
            v[u] = k0 + u < e ? vv : 0.0;
        }
        double xv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) xv[u] = x[(uint32_t)c[u]];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (k0 + u < e) acc += v[u] * xv[u];
    }
    double r = alpha * acc;
    if (beta != 0.0) r += beta * zr;
    y[row] = r;
}

// Long rows (mean >= 96 nnz): one wave walks `rpw` consecutive rows two at a
// time; for each row pair all U*64 val/col loads per row are issued before the
// x gathers, so a wave keeps ~4.6 KB of HBM loads in flight (the one-row-per-
// wave form is latency bound at ~2 TB/s).
template <int U>
__global__ __launch_bounds__(TPB) void k_spmv_w64(int64_t nrows, int rpw, const int64_t *__restrict__ rp,
                                                  const int32_t *__restrict__ ci, const double *__restrict__ val,
                                                  const double *__restrict__ x, double *__restrict__ y,
                                                  double alpha, double beta, const double *__restrict__ z) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (TPB / 64) + (threadIdx.x >> 6)));
    const int64_t r0 = (int64_t)wave * rpw;
    if (r0 >= nrows) return;
    const int64_t r1 = (r0 + rpw < nrows) ? r0 + rpw : nrows;
    for (int64_t r = r0; r < r1; r += 2) {
        const bool two = (r + 1 < r1);
        const int64_t sa = rp[r], ea = rp[r + 1];
        const int64_t eb = two ? rp[r + 2] : ea;
        double acc_a = 0.0, acc_b = 0.0;
        for (int64_t ka = sa, kb = ea; ka < ea || kb < eb; ka += U * 64, kb += U * 64) {
            int32_t ca[U], cb[U];
            double va[U], vb[U];
// unconditional loads at a clamped index (entry 0 is always valid), value
            // masked to 0: no exec-masked branch, so all 4U loads issue back to back
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t k = ka + u * 64 + lane;
                const int64_t kk = k < ea ? k : 0;
                ca[u] = __builtin_nontemporal_load(ci + kk);
                const double v = __builtin_nontemporal_load(val + kk);
                va[u] = k < ea ? v : 0.0;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t k = kb + u * 64 + lane;
                const int64_t kk = k < eb ? k : 0;
                cb[u] = __builtin_nontemporal_load(ci + kk);
                const double v = __builtin_nontemporal_load(val + kk);
                vb[u] = k < eb ? v : 0.0;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                acc_a += va[u] * x[(uint32_t)ca[u]];
                acc_b += vb[u] * x[(uint32_t)cb[u]];
            }
        }
        acc_a = wave_reduce(acc_a);
        acc_b = wave_reduce(acc_b);
        if (lane == 0) {
            double ra = alpha * acc_a;
            if (beta != 0.0) ra += beta * z[r];
            y[r] = ra;
            if (two) {
                double rb = alpha * acc_b;
                if (beta != 0.0) rb += beta * z[r + 1];
                y[r + 1] = rb;
            }
        }
    }
}

// Few, very long rows (AMG restriction R = P^T, Galerkin coarse operators,
// the dense coarsest inverse): one 256-lane workgroup per row, U loads per
// lane in flight, fixed-order wave + LDS reduction (deterministic).
template <int U>
__global__ __launch_bounds__(TPB) void k_spmv_wg(int64_t nrows, const int64_t *__restrict__ rp,
                                                 const int32_t *__restrict__ ci, const double *__restrict__ val,
                                                 const double *__restrict__ x, double *__restrict__ y, double alpha,
                                                 double beta, const double *__restrict__ z) {
    __shared__ double part[TPB / 64];
    const int64_t row = blockIdx.x;
    const int64_t s = rp[row], e = rp[row + 1];
    double acc = 0.0;
    for (int64_t k0 = s; k0 < e; k0 += U * TPB) {
        int32_t c[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t k = k0 + u * TPB + threadIdx.x;
            const int64_t kk = k < e ? k : s;
            c[u] = __builtin_nontemporal_load(ci + kk);
            const double vv = __builtin_nontemporal_load(val + kk);
            v[u] = k < e ? vv : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u] * x[(uint32_t)c[u]];
    }
    acc = wave_reduce(acc);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = part[0];
#pragma unroll
        for (int w = 1; w < TPB / 64; ++w) t += part[w];
        double r = alpha * t;
        if (beta != 0.0) r += beta * z[row];
        y[row] = r;
    }
}

static bool spmv_short_rows = false;
void set_spmv_short_rows(bool on) { spmv_short_rows = on; }

void launch_spmv(int64_t nrows, int64_t nnz, const int64_t *rp, const int32_t *ci, const double *val,
                 const double *x, double *y, double alpha, double beta, const double *z, hipStream_t st) {
    if (nrows <= 0) return;
    const double mean = (double)nnz / (double)nrows;
    if (mean >= 512.0 || (mean >= 96.0 && nrows < 16384)) {
        k_spmv_wg<4><<<(unsigned)nrows, TPB, 0, st>>>(nrows, rp, ci, val, x, y, alpha, beta, z);
    } else if (mean >= 96.0) {
        const int rpw = 8;
        const int64_t waves = (nrows + rpw - 1) / rpw;
        k_spmv_w64<3><<<grid_for(waves, TPB / 64), TPB, 0, st>>>(nrows, rpw, rp, ci, val, x, y, alpha, beta, z);
    } else if (mean >= 40.0)
        k_spmv<32><<<grid_for(nrows, TPB / 32), TPB, 0, st>>>(nrows, rp, ci, val, x, y, alpha, beta, z);
    else if (mean >= 16.0)
        k_spmv<16><<<grid_for(nrows, TPB / 16), TPB, 0, st>>>(nrows, rp, ci, val, x, y, alpha, beta, z);
    else if (mean >= 12.0 || !spmv_short_rows)
        k_spmv<8><<<grid_for(nrows, TPB / 8), TPB, 0, st>>>(nrows, rp, ci, val, x, y, alpha, beta, z);
    else
        k_spmv_short<<<grid_for(nrows, TPB), TPB, 0, st>>>(nrows, rp, ci, val, x, y, alpha, beta, z);
}

// =============================================================== BLAS-1 ====
__global__ __launch_bounds__(TPB) void k_copy(int64_t n, const double *x, double *y) {
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) y[i] = x[i];
}
__global__ __launch_bounds__(TPB) void k_set(int64_t n, double a, double *y) {
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) y[i] = a;
}
__global__ __launch_bounds__(TPB) void k_scale(int64_t n, double a, double *y) {
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) y[i] *= a;
}
// (pa / pb: the scalars read from device memory instead, skip: no-op when *skip
// -- the device-resident CG; one kernel body, so both paths round alike)
__global__ __launch_bounds__(TPB) void k_axpby(int64_t n, double a, const double *x, double b, double *y,
                                               const double *pa, const double *pb, const int64_t *skip) {
    if (skip && *skip) return;
    if (pa) a = *pa;
    if (pb) b = *pb;
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB)
        y[i] = a * x[i] + b * y[i];
}
__global__ __launch_bounds__(TPB) void k_waxpby(int64_t n, double a, const double *x, double b,
                                                const double *y, double *w) {
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB)
        w[i] = a * x[i] + b * y[i];
}
__global__ __launch_bounds__(TPB) void k_pmult(int64_t n, const double *x, const double *d, double *y) {
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB)
        y[i] = x[i] * d[i];
}
__global__ __launch_bounds__(TPB) void k_zero_entries(int64_t m, const int32_t *idx, double *y) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i < m) y[idx[i]] = 0.0;
}
__global__ __launch_bounds__(TPB) void k_gather(int64_t n, const int64_t *idx, const double *x, double *y) {
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB)
        y[i] = x[idx[i]];
}
__global__ __launch_bounds__(TPB) void k_scatter(int64_t n, const int64_t *idx, const double *x, double *y) {
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB)
        y[idx[i]] = x[i];
}

// AMG Chebyshev/Jacobi step (oracle/amg.py PCAMG._cheb), fused:
// d = a d + bc (dinv . r), x += d;  flags 1: d not read (d = bc (dinv . r)),
// flags 2: x not read (x = d)
__global__ __launch_bounds__(TPB) void k_cheb_step(int64_t n, const double *__restrict__ dinv,
                                                   const double *__restrict__ r, double *__restrict__ d,
                                                   double *__restrict__ x, double a, double bc, int flags) {
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
        const double t = dinv[i] * r[i];
        const double dn = (flags & 1) ? bc * t : a * d[i] + bc * t;
        d[i] = dn;
        x[i] = (flags & 2) ? dn : x[i] + dn;
    }
}

static inline unsigned stream_grid(int64_t n) {
    int64_t g = (n + TPB - 1) / TPB;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    return (unsigned)g;
}

// streaming probes (the achievable HBM rate): 16 B per lane,
// four loads in flight per lane, nontemporal.  mode 0: copy (read + write),
// mode 1: read-only (the SpMV's traffic mix is ~99 % reads)
typedef double probe_d2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(TPB) void k_copy_probe(int64_t n2, const probe_d2 *__restrict__ x,
                                                    probe_d2 *__restrict__ y, int mode, double *sink) {
    const int64_t stride = (int64_t)gridDim.x * TPB;
    probe_d2 acc = {0.0, 0.0};
    for (int64_t i0 = (int64_t)blockIdx.x * TPB + threadIdx.x; i0 < n2; i0 += 4 * stride) {
        probe_d2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = i0 + u * stride;
            v[u] = i < n2 ? __builtin_nontemporal_load(x + i) : probe_d2{0.0, 0.0};
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = i0 + u * stride;
            if (mode == 0) {
                if (i < n2) __builtin_nontemporal_store(v[u], y + i);
            } else {
                acc += v[u];
            }
        }
    }
    if (mode == 1 && acc.x + acc.y == 12345.678) sink[0] = acc.x;
}
void launch_copy_probe(int64_t n, const double *x, double *y, int mode, hipStream_t st) {
    if (n > 1)
        k_copy_probe<<<8192, TPB, 0, st>>>(n / 2, reinterpret_cast<const probe_d2 *>(x), reinterpret_cast<probe_d2 *>(y),
                                            mode, y);
}
void launch_copy(int64_t n, const double *x, double *y, hipStream_t st) {
    if (n > 0) k_copy<<<stream_grid(n), TPB, 0, st>>>(n, x, y);
}
void launch_set(int64_t n, double a, double *y, hipStream_t st) {
    if (n > 0) k_set<<<stream_grid(n), TPB, 0, st>>>(n, a, y);
}
void launch_scale(int64_t n, double a, double *y, hipStream_t st) {
    if (n > 0) k_scale<<<stream_grid(n), TPB, 0, st>>>(n, a, y);
}
void launch_axpby(int64_t n, double a, const double *x, double b, double *y, hipStream_t st) {
    if (n > 0) k_axpby<<<stream_grid(n), TPB, 0, st>>>(n, a, x, b, y, nullptr, nullptr, nullptr);
}
void launch_axpby_dev(int64_t n, const double *pa, const double *x, const double *pb, double *y, const int64_t *skip,
                      hipStream_t st) {
    if (n > 0) k_axpby<<<stream_grid(n), TPB, 0, st>>>(n, 0.0, x, 0.0, y, pa, pb, skip);
}

// ------------------------------------------------ device-resident CG state --
// KSPSolve_CG's scalar recurrences (runtime.cpp KSP::solve_cg) on the device,
// one thread, so the host enqueues iterations without reading a scalar back:
// every phase returns at once when the solve has ended (I[CG_DONE]); the
// vector updates that follow check the same flag.  Same operations as the host
// loop (IEEE division and square root): bitwise the same iterates.
__device__ int cg_conv(const CgParams &p, double r, double rnorm0, double ttol) {
    if (isnan(r) || isinf(r)) return p.r_nan;
    if (r <= ttol) return r < p.atol ? p.r_atol : p.r_rtol;
    if (r >= p.dtol * rnorm0) return p.r_dtol;
    return 0;
}
__global__ void k_cg_state(int phase, int64_t i, double *S, int64_t *I, double *hist, CgParams p) {
    if (threadIdx.x != 0 || I[CG_DONE]) return;
    auto stop = [&](int reason) {
        I[CG_REASON] = reason;
        I[CG_DONE] = 1;
    };
    switch (phase) {
        case CG_TOP: {  // loop head of iteration i (beta = (z, r) of the previous step)
            I[CG_ITS] = i + 1;
            const double beta = S[CG_BETA], betaold = S[CG_BETAOLD];
            if (beta == 0.0) return stop(p.r_atol);
            if (i > 0 && beta * betaold < 0.0) return stop(p.r_indef_pc);
            if (i > 0) S[CG_BB] = beta / betaold;
            return;
        }
        case CG_MID: {  // dpi = (p, A p) in S[CG_SLOT]
            const double dpiold = S[CG_DPI], dpi = S[CG_SLOT];
            S[CG_DPI] = dpi;
            S[CG_BETAOLD] = S[CG_BETA];
            const int sd = (dpi > 0) - (dpi < 0), so = (dpiold > 0) - (dpiold < 0);
            if (dpi == 0.0 || (i > 0 && sd * so < 0)) return stop(p.r_indef_mat);
            const double a = S[CG_BETA] / dpi;
            S[CG_A] = a;
            S[CG_NEGA] = -a;
            return;
        }
        case CG_POST: {  // the residual norm's square (or 0) in S[CG_SLOT]
            const double dp = p.norm ? sqrt(S[CG_SLOT]) : 0.0;
            S[CG_RNORM] = dp;
            hist[I[CG_HCOUNT]++] = dp;
            if (p.norm) {
                const int r = cg_conv(p, dp, S[CG_RNORM0], S[CG_TTOL]);
                if (r) return stop(r);
            }
            return;
        }
        case CG_END: {  // beta = (z, r) in S[CG_SLOT2]; i counts this iteration
            S[CG_BETA] = S[CG_SLOT2];
            if (i + 1 >= p.maxit) return stop(p.r_its);
            return;
        }
    }
}
void launch_cg_state(int phase, int64_t i, double *S, int64_t *I, double *hist, const CgParams &p, hipStream_t st) {
    k_cg_state<<<1, 64, 0, st>>>(phase, i, S, I, hist, p);
}
void launch_waxpby(int64_t n, double a, const double *x, double b, const double *y, double *w, hipStream_t st) {
    if (n > 0) k_waxpby<<<stream_grid(n), TPB, 0, st>>>(n, a, x, b, y, w);
}
void launch_pointwise_mult(int64_t n, const double *x, const double *d, double *y, hipStream_t st) {
    if (n > 0) k_pmult<<<stream_grid(n), TPB, 0, st>>>(n, x, d, y);
}
void launch_cheb_step(int64_t n, const double *dinv, const double *r, double *d, double *x, double a, double bc,
                      int flags, hipStream_t st) {
    if (n > 0) k_cheb_step<<<stream_grid(n), TPB, 0, st>>>(n, dinv, r, d, x, a, bc, flags);
}
void launch_zero_entries(int64_t m, const int32_t *idx, double *y, hipStream_t st) {
    if (m > 0) k_zero_entries<<<grid_for(m, TPB), TPB, 0, st>>>(m, idx, y);
}
void launch_gather(int64_t n, const int64_t *idx, const double *x, double *y, hipStream_t st) {
    if (n > 0) k_gather<<<stream_grid(n), TPB, 0, st>>>(n, idx, x, y);
}
void launch_scatter(int64_t n, const int64_t *idx, const double *x, double *y, hipStream_t st) {
    if (n > 0) k_scatter<<<stream_grid(n), TPB, 0, st>>>(n, idx, x, y);
}

// ---------------------------------------------- deterministic reductions --
// up to 4096 blocks (16 waves per CU): with 1024 the multi-vector CGS
// kernels (k_mdot / k_maxpy_norm) held 4 waves per CU and read the Krylov
// basis at ~2.8 TB/s (profiles/r04_hyp59)
static constexpr int NB_MAX = 4096;
int reduce_blocks(int64_t n) {
    int64_t nb = (n + 4095) / 4096;
    if (nb < 1) nb = 1;
    if (nb > NB_MAX) nb = NB_MAX;
    return (int)nb;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
// fixed-order block reduction (TPB threads); result valid in thread 0
__device__ __forceinline__ double block_sum(double v, double *lds) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) lds[w] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < TPB / 64; ++i) r += lds[i];
    }
    __syncthreads();
    return r;
}

__device__ __forceinline__ void chunk_of(int64_t n, int nb, int b, int64_t &s, int64_t &e) {
    const int64_t c = (n + nb - 1) / nb;
    s = (int64_t)b * c;
    e = s + c;
    if (e > n) e = n;
    if (s > n) s = n;
}

// final pass: out[j] = sum_b partial[j*nb + b]
__global__ __launch_bounds__(TPB) void k_final(int nb, const double *partial, double *out, int sqrt_it) {
    __shared__ double lds[TPB / 64];
    const int j = blockIdx.x;
    double v = 0.0;
    for (int b = threadIdx.x; b < nb; b += TPB) v += partial[(int64_t)j * nb + b];
    v = block_sum(v, lds);
    if (threadIdx.x == 0) out[j] = sqrt_it ? sqrt(v) : v;
}

// mdot: blockIdx.x = chunk, blockIdx.y = group of MDOT_NJ vectors
// CGS dot block h_j = V_j . w, j in [0, k): blocks of MDOT_NJ columns per
// grid row, 16-B loads (pairs of rows; chunks start on even rows, V columns
// are 512-B aligned), one partial per (column, block) -> k_final in fixed order.
typedef double cgs_d2 __attribute__((ext_vector_type(2)));
static constexpr int MDOT_NJ = 16;
__device__ __forceinline__ void chunk_even(int64_t n, int nb, int b, int64_t &s, int64_t &e) {
    int64_t c = (n + nb - 1) / nb;
    c = (c + 1) & ~(int64_t)1;
    s = (int64_t)b * c;
    e = s + c;
    if (e > n) e = n;
    if (s > n) s = n;
}
__global__ __launch_bounds__(TPB) void k_mdot(int64_t n, int k, const double *__restrict__ V, int64_t ldv,
                                              const double *__restrict__ w, double *partial) {
    __shared__ double lds[TPB / 64];
    const int nb = gridDim.x;
    int64_t s, e;
    chunk_even(n, nb, blockIdx.x, s, e);
    const int j0 = blockIdx.y * MDOT_NJ;
    const int nj = (k - j0) < MDOT_NJ ? (k - j0) : MDOT_NJ;
    double a[MDOT_NJ];
#pragma unroll
    for (int u = 0; u < MDOT_NJ; ++u) a[u] = 0.0;
    const double *v0 = V + (int64_t)j0 * ldv;
    int64_t i = s + 2 * threadIdx.x;
    // two row pairs per trip, all their loads issued before the FMAs (twice the
    // bytes in flight; the same per-thread summation order as one pair a trip)
    for (; i + 2 * TPB + 1 < e; i += 4 * TPB) {
        const cgs_d2 wa = *reinterpret_cast<const cgs_d2 *>(w + i);
        const cgs_d2 wb = *reinterpret_cast<const cgs_d2 *>(w + i + 2 * TPB);
        cgs_d2 va[MDOT_NJ], vb[MDOT_NJ];
#pragma unroll
        for (int u = 0; u < MDOT_NJ; ++u) {
            if (u < nj) {
                va[u] = *reinterpret_cast<const cgs_d2 *>(v0 + (int64_t)u * ldv + i);
                vb[u] = *reinterpret_cast<const cgs_d2 *>(v0 + (int64_t)u * ldv + i + 2 * TPB);
            }
        }
#pragma unroll
        for (int u = 0; u < MDOT_NJ; ++u) {
            if (u < nj) {
                a[u] += va[u].x * wa.x;
                a[u] += va[u].y * wa.y;
                a[u] += vb[u].x * wb.x;
                a[u] += vb[u].y * wb.y;
            }
        }
    }
    for (; i + 1 < e; i += 2 * TPB) {
        const cgs_d2 wi = *reinterpret_cast<const cgs_d2 *>(w + i);
#pragma unroll
        for (int u = 0; u < MDOT_NJ; ++u) {
            if (u < nj) {
                const cgs_d2 v = *reinterpret_cast<const cgs_d2 *>(v0 + (int64_t)u * ldv + i);
                a[u] += v.x * wi.x;
                a[u] += v.y * wi.y;
            }
        }
    }
    if (((e - s) & 1) && threadIdx.x == 0) {
        const int64_t i = e - 1;
#pragma unroll
        for (int u = 0; u < MDOT_NJ; ++u)
            if (u < nj) a[u] += v0[(int64_t)u * ldv + i] * w[i];
    }
#pragma unroll
    for (int u = 0; u < MDOT_NJ; ++u) {
        if (u < nj) {
            const double r = block_sum(a[u], lds);
            if (threadIdx.x == 0) partial[(int64_t)(j0 + u) * nb + blockIdx.x] = r;
        }
    }
}

void launch_mdot(int64_t n, int k, const double *const *, const double *V, int64_t ldv, const double *w,
                 double *partial, double *out, hipStream_t st) {
    if (k <= 0) return;
    const int nb = reduce_blocks(n);
    dim3 grid(nb, (k + MDOT_NJ - 1) / MDOT_NJ);
    k_mdot<<<grid, TPB, 0, st>>>(n, k, V, ldv, w, partial);
    k_final<<<k, TPB, 0, st>>>(nb, partial, out, 0);
}

__global__ __launch_bounds__(TPB) void k_dot(int64_t n, const double *__restrict__ x, const double *__restrict__ y,
                                             double *partial) {
    __shared__ double lds[TPB / 64];
    int64_t s, e;
    chunk_of(n, gridDim.x, blockIdx.x, s, e);
    double a = 0.0;
    for (int64_t i = s + threadIdx.x; i < e; i += TPB) a += x[i] * y[i];
    a = block_sum(a, lds);
    if (threadIdx.x == 0) partial[blockIdx.x] = a;
}

void launch_dot(int64_t n, const double *x, const double *y, double *partial, double *out, hipStream_t st) {
    const int nb = reduce_blocks(n);
    k_dot<<<nb, TPB, 0, st>>>(n, x, y, partial);
    k_final<<<1, TPB, 0, st>>>(nb, partial, out, 0);
}
void launch_norm2(int64_t n, const double *x, double *partial, double *out, hipStream_t st) {
    const int nb = reduce_blocks(n);
    k_dot<<<nb, TPB, 0, st>>>(n, x, x, partial);
    k_final<<<1, TPB, 0, st>>>(nb, partial, out, 1);
}

// w -= sum_j h[j] V[:, j] (j ascending, as VecMAXPY); partial ||w||^2.
// Pairs of rows per thread (16-B loads), eight basis columns loaded ahead of
// their FMAs so every lane keeps 8-9 loads in flight.
__global__ __launch_bounds__(TPB) void k_maxpy_norm(int64_t n, int k, const double *__restrict__ V, int64_t ldv,
                                                    const double *__restrict__ h, double *__restrict__ w,
                                                    double *partial) {
    __shared__ double lds[TPB / 64];
    __shared__ double hs[512];
    for (int j = threadIdx.x; j < k && j < 512; j += TPB) hs[j] = h[j];
    __syncthreads();
    int64_t s, e;
    chunk_even(n, gridDim.x, blockIdx.x, s, e);
    double a = 0.0;
    int64_t i = s + 2 * threadIdx.x;
    // two row pairs per trip (loads of both ahead of their FMAs; the norm sums
    // the pairs in the same order as one pair a trip)
    for (; i + 2 * TPB + 1 < e; i += 4 * TPB) {
        cgs_d2 ta = *reinterpret_cast<const cgs_d2 *>(w + i);
        cgs_d2 tb = *reinterpret_cast<const cgs_d2 *>(w + i + 2 * TPB);
        int j = 0;
        for (; j + 8 <= k; j += 8) {
            cgs_d2 va[8], vb[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                va[u] = *reinterpret_cast<const cgs_d2 *>(V + (int64_t)(j + u) * ldv + i);
                vb[u] = *reinterpret_cast<const cgs_d2 *>(V + (int64_t)(j + u) * ldv + i + 2 * TPB);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const double hj = (j + u) < 512 ? hs[j + u] : h[j + u];
                ta.x -= hj * va[u].x;
                ta.y -= hj * va[u].y;
                tb.x -= hj * vb[u].x;
                tb.y -= hj * vb[u].y;
            }
        }
        for (; j < k; ++j) {
            const cgs_d2 va = *reinterpret_cast<const cgs_d2 *>(V + (int64_t)j * ldv + i);
            const cgs_d2 vb = *reinterpret_cast<const cgs_d2 *>(V + (int64_t)j * ldv + i + 2 * TPB);
            const double hj = j < 512 ? hs[j] : h[j];
            ta.x -= hj * va.x;
            ta.y -= hj * va.y;
            tb.x -= hj * vb.x;
            tb.y -= hj * vb.y;
        }
        *reinterpret_cast<cgs_d2 *>(w + i) = ta;
        *reinterpret_cast<cgs_d2 *>(w + i + 2 * TPB) = tb;
        a += ta.x * ta.x;
        a += ta.y * ta.y;
        a += tb.x * tb.x;
        a += tb.y * tb.y;
    }
    for (; i + 1 < e; i += 2 * TPB) {
        cgs_d2 t = *reinterpret_cast<const cgs_d2 *>(w + i);
        int j = 0;
        for (; j + 8 <= k; j += 8) {
            cgs_d2 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const cgs_d2 *>(V + (int64_t)(j + u) * ldv + i);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const double hj = (j + u) < 512 ? hs[j + u] : h[j + u];
                t.x -= hj * v[u].x;
                t.y -= hj * v[u].y;
            }
        }
        for (; j < k; ++j) {
            const cgs_d2 v = *reinterpret_cast<const cgs_d2 *>(V + (int64_t)j * ldv + i);
            const double hj = j < 512 ? hs[j] : h[j];
            t.x -= hj * v.x;
            t.y -= hj * v.y;
        }
        *reinterpret_cast<cgs_d2 *>(w + i) = t;
        a += t.x * t.x;
        a += t.y * t.y;
    }
    if (((e - s) & 1) && threadIdx.x == 0) {
        const int64_t i = e - 1;
        double t = w[i];
        for (int j = 0; j < k; ++j) t -= (j < 512 ? hs[j] : h[j]) * V[(int64_t)j * ldv + i];
        w[i] = t;
        a += t * t;
    }
    if (partial) {
        a = block_sum(a, lds);
        if (threadIdx.x == 0) partial[blockIdx.x] = a;
    }
}

void launch_maxpy_norm(int64_t n, int k, const double *V, int64_t ldv, const double *h_dev, double,
                       double *w, double *partial, double *out, hipStream_t st) {
    const int nb = reduce_blocks(n);
    k_maxpy_norm<<<nb, TPB, 0, st>>>(n, k, V, ldv, h_dev, w, out ? partial : nullptr);
    if (out) k_final<<<1, TPB, 0, st>>>(nb, partial, out, 0);  // ||w||^2 (rank-local)
}

__global__ __launch_bounds__(TPB) void k_lincomb(int64_t n, int k, const double *__restrict__ V, int64_t ldv,
                                                 const double *__restrict__ c, double *__restrict__ y) {
    __shared__ double cs[512];
    for (int j = threadIdx.x; j < k && j < 512; j += TPB) cs[j] = c[j];
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
        double t = 0.0;
        for (int j = 0; j < k; ++j) t += (j < 512 ? cs[j] : c[j]) * V[(int64_t)j * ldv + i];
        y[i] = t;
    }
}
void launch_lincomb(int64_t n, int k, const double *V, int64_t ldv, const double *c_dev, double *y,
                    hipStream_t st) {
    if (n > 0) k_lincomb<<<stream_grid(n), TPB, 0, st>>>(n, k, V, ldv, c_dev, y);
}

// TSQR leaf / tree step for the Anderson least squares (numpy Householder QR
// in the reference, lib/AAR.py:102-105): workgroup b takes rows
// [b C, b C + C) of the m <= 16 columns cols[k] (rows >= n read as zero),
// factors that C x m panel in LDS by m Householder reflections (LAPACK dlarfg
// conventions: beta = -sign(alpha) ||x||, tau = (beta - alpha) / beta,
// v = x / (alpha - beta) below the diagonal) and writes its m x m R (zero
// below the diagonal) as rows [b m, b m + m) of a column-major matrix with
// leading dimension ldo.  Stacked R's are factored again by the same kernel
// until one R is left (a fixed tree: bitwise reproducible).  Each reflection
// is one block reduction of the m - j dots sum_{r>j} A[j][r] A[k][r] (fixed
// order: per-thread rows ascending, xor-shuffle tree, 4 waves in order).
constexpr int TSQR_C = 512;
template <int M>
__global__ __launch_bounds__(256) void k_tsqr(int64_t n, const double *const *cols, double *Rout, int64_t ldo) {
    constexpr int C = TSQR_C, RPT = C / 256;
    __shared__ double A[M * C];
    __shared__ double red[4][M];
    __shared__ double w[M];
    __shared__ double cf[3];  // tau, scal, beta
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t r0 = (int64_t)blockIdx.x * C;
#pragma unroll
    for (int k = 0; k < M; ++k) {
        const double *cp = cols[k];
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int r = tid + q * 256;
            const int64_t g = r0 + r;
            A[k * C + r] = g < n ? cp[g] : 0.0;
        }
    }
    __syncthreads();
    for (int j = 0; j < M; ++j) {
        double p[M];
#pragma unroll
        for (int k = 0; k < M; ++k) p[k] = 0.0;
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int r = tid + q * 256;
            if (r > j) {
                const double vj = A[j * C + r];
#pragma unroll
                for (int k = 0; k < M; ++k)
                    if (k >= j) p[k] += vj * A[k * C + r];
            }
        }
#pragma unroll
        for (int k = 0; k < M; ++k) {
            if (k < j) continue;
            double v = p[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) red[wv][k] = v;
        }
        __syncthreads();
        if (tid < M) {
            const double sigma = ((red[0][j] + red[1][j]) + red[2][j]) + red[3][j];
            const double alpha = A[j * C + j];
            double tau = 0.0, scal = 0.0, beta = alpha;
            if (sigma != 0.0) {
                const double nrm = sqrt(alpha * alpha + sigma);
                beta = alpha >= 0.0 ? -nrm : nrm;
                tau = (beta - alpha) / beta;
                scal = 1.0 / (alpha - beta);
            }
            if (tid > j) {
                const double sk = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
                w[tid] = A[tid * C + j] + scal * sk;
            }
            if (tid == 0) { cf[0] = tau; cf[1] = scal; cf[2] = beta; }
        }
        __syncthreads();
        const double tau = cf[0], scal = cf[1];
        if (tau != 0.0) {
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
                const int r = tid + q * 256;
                if (r > j) {
                    const double v = A[j * C + r] * scal;
#pragma unroll
                    for (int k = 0; k < M; ++k)
                        if (k > j) A[k * C + r] -= tau * w[k] * v;
                } else if (r == j) {
#pragma unroll
                    for (int k = 0; k < M; ++k)
                        if (k > j) A[k * C + j] -= tau * w[k];
                }
            }
        }
        if (tid == j) A[j * C + j] = cf[2];
        __syncthreads();
    }
    for (int t = tid; t < M * M; t += 256) {
        const int k = t / M, i = t % M;
        Rout[(int64_t)k * ldo + (int64_t)blockIdx.x * M + i] = i <= k ? A[k * C + i] : 0.0;
    }
}

int tsqr_rows_per_block() { return TSQR_C; }

void launch_tsqr(int64_t n, int m, const double *const *cols_dev, double *Rout, int64_t ldo, hipStream_t st) {
    const unsigned nb = (unsigned)((n + TSQR_C - 1) / TSQR_C);
    if (nb == 0) return;
    switch (m) {
#define PLS_TSQR(M) case M: k_tsqr<M><<<nb, 256, 0, st>>>(n, cols_dev, Rout, ldo); break;
        PLS_TSQR(1) PLS_TSQR(2) PLS_TSQR(3) PLS_TSQR(4) PLS_TSQR(5) PLS_TSQR(6) PLS_TSQR(7) PLS_TSQR(8)
        PLS_TSQR(9) PLS_TSQR(10) PLS_TSQR(11) PLS_TSQR(12) PLS_TSQR(13) PLS_TSQR(14) PLS_TSQR(15) PLS_TSQR(16)
#undef PLS_TSQR
        default: return;
    }
}

// ================================================================ ILU(0) ===
__global__ __launch_bounds__(TPB) void k_find_diag(int64_t n, const int64_t *rp, const int32_t *ci,
                                                   int64_t *diag, int32_t *fail) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    const int64_t p = lower_bound_i32(ci, rp[i], rp[i + 1], i);
    if (p < rp[i + 1] && (int64_t)ci[p] == i) {
        diag[i] = p;
    } else {
        diag[i] = -1;
        atomicMax(fail, 1);
    }
}
void launch_find_diag(int64_t n, const int64_t *rp, const int32_t *ci, int64_t *diag, int32_t *fail,
                      hipStream_t st) {
    if (n > 0) k_find_diag<<<grid_for(n, TPB), TPB, 0, st>>>(n, rp, ci, diag, fail);
}

// Symmetric Gauss-Seidel factors (see kernels.hpp): 1/a_ii first, then every
// strict-lower entry a_ij -> a_ij * (1/a_jj), the multiplier the ILU(0) IKJ
// loop forms (k_ilu0_level: mult = a_ij * dinv[j]).
__global__ __launch_bounds__(TPB) void k_sgs_dinv(int64_t n, const double *lu, const int64_t *diag, double *dinv,
                                                  int32_t *fail) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    const double d = lu[diag[i]];
    if (d == 0.0) {
        atomicMax(fail, 2);
        dinv[i] = 0.0;
    } else {
        dinv[i] = 1.0 / d;
    }
}
__global__ __launch_bounds__(TPB) void k_sgs_scale(int64_t n, const int64_t *rp, const int32_t *ci, double *lu,
                                                   const int64_t *diag, const double *dinv) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    for (int64_t k = rp[i]; k < diag[i]; ++k) lu[k] = lu[k] * dinv[ci[k]];
}
void launch_sgs_factor(int64_t n, const int64_t *rp, const int32_t *ci, double *lu, const int64_t *diag,
                       double *dinv, int32_t *fail, hipStream_t st) {
    if (n <= 0) return;
    k_sgs_dinv<<<grid_for(n, TPB), TPB, 0, st>>>(n, lu, diag, dinv, fail);
    k_sgs_scale<<<grid_for(n, TPB), TPB, 0, st>>>(n, rp, ci, lu, diag, dinv);
}

// ILU(0) numeric factorization, one workgroup (ILU0_TPB threads) per row.
// The row is staged in LDS (values, columns and a column -> position hash);
// the upper parts of its pivot rows (rows r of earlier levels, final) and
// their 1/u_rr are staged in LDS too, in segments of at most ILU0_STAGE
// entries -- all four waves' loads in flight at once -- and every staged
// entry's position in the row is resolved while staging (the hash probes do
// not depend on the elimination).  Wave 0 then runs the IKJ elimination over
// the row's strict-lower entries in column order with the next pivot's
// positions and values prefetched, so a pivot step is one LDS round trip
// (rv[t] and the entries it updates) plus the update.  A pivot whose upper
// part alone exceeds the stage reads global memory.  Same operations in the
// same order as the CPU restatement (no contraction): bitwise the same
// factors whatever the path.
// DEP (k_ilu0_dep): one persistent launch -- rows are drawn from a counter in
// level order and each waits for its pivot rows' completion flags.  Pivot
// data written by other workgroups is read with agent-coherent (sc1) loads
// and the row's results are written with agent-coherent stores, so neither
// side needs the L2 write-back / invalidate of a release / acquire fence
// (one per row measured ~1.8x slower rows: every row's fence emptied the
// XCD's L2 for all the others).
static constexpr int ILU0_TPB = 256;
static constexpr int ILU0_STAGE = 8192;  // staged upper-part entries per segment (96 KiB)
__constant__ int ilu0_probe;  // diagnostics (pls.ilu0_probe N): phase times of every N-th row to stdout
void set_ilu0_probe(int v) { (void)hipMemcpyToSymbol(HIP_SYMBOL(ilu0_probe), &v, sizeof(int)); }
static constexpr int64_t ILU0_SPIN_MAX = 1ll << 24;  // dependency polls before a row gives up (never expected)
static constexpr int ILU0_LDS = 163840 - 512;         // dynamic LDS budget (beside ilu0_ctl, ilu0_cnt)
__shared__ int32_t ilu0_ctl[4];                       // [0] drawn row (DEP), [1] abort
__shared__ int32_t ilu0_cnt[64];                      // per pivot chunk: staging waves done (DEP)

template <bool COH>
__device__ __forceinline__ double ilu0_ld(const double *p) {
    if (COH)
        return __longlong_as_double((long long)__hip_atomic_load(
            reinterpret_cast<uint64_t *>(const_cast<double *>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    return *p;
}
template <bool COH>
__device__ __forceinline__ void ilu0_st(double *p, double v) {
    if (COH)
        __hip_atomic_store(reinterpret_cast<uint64_t *>(p), (uint64_t)__double_as_longlong(v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}

// stage pivots [ta, tb)'s upper parts (entries so[t] - base ..): POS their
// positions in the row (sc), VAL their values (sv); eight loads per thread in
// flight, entry q's pivot found by binary search over so
template <bool COH, bool POS, bool VAL>
__device__ __forceinline__ void ilu0_stage_part(int ta, int tb, int base, int cnt, const int64_t *__restrict__ rp,
                                                const int32_t *__restrict__ ci, const double *lu, int len, int hbits,
                                                const int32_t *rc, const int32_t *so, const int64_t *su, int32_t *sc,
                                                double *sv, const int32_t *hk, const int32_t *hp, int wbase = 0,
                                                int tid_ = -1, int nthr = ILU0_TPB) {
    // (entry base + q is written at wbase + q; threads tid_ of nthr, default all)
    const int tid = tid_ < 0 ? (int)threadIdx.x : tid_;
    const uint32_t hmask = (1u << hbits) - 1;
    for (int q0 = 0; q0 < cnt; q0 += 8 * nthr) {
        int64_t src[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = base + q0 + u * nthr + tid;
            int lo = ta, hi = tb;  // last t with so[t] <= q
            while (hi - lo > 1) {
                const int m = (lo + hi) >> 1;
                if (so[m] <= q) lo = m; else hi = m;
            }
            src[u] = q < base + cnt ? su[lo] + (q - so[lo]) : su[ta];
        }
        int32_t cv[8];
        double vv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (POS) cv[u] = ci[src[u]];
            if (VAL) vv[u] = ilu0_ld<COH>(lu + src[u]);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = q0 + u * nthr + tid;
            if (q < cnt) {
                if (POS) {  // the column's position in the row (len: not in the pattern)
                    const int32_t j = cv[u];
                    int lo = len;
                    if (hbits > 0) {
                        uint32_t h = ((uint32_t)j * 2654435761u) >> (32 - hbits);
                        int32_t key = hk[h];
                        while (key != j && key != -1) {
                            h = (h + 1) & hmask;
                            key = hk[h];
                        }
                        if (key == j) lo = hp[h];
                    } else {
                        int a = 0, b = len;
                        while (a < b) {
                            const int m = (a + b) >> 1;
                            if (rc[m] < j) a = m + 1; else b = m;
                        }
                        if (a < len && rc[a] == j) lo = a;
                    }
                    sc[wbase + q] = lo;
                }
                if (VAL) sv[wbase + q] = vv[u];
            }
        }
    }
}

#pragma clang fp contract(off)
// returns false when the launch aborts (DEP: a dependency wait exceeded its bound)
template <bool DEP>
__device__ __forceinline__ bool ilu0_row(int64_t i, const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                         double *lu, const int64_t *__restrict__ diag, double *dinv, int32_t *fail,
                                         int max_row, int stage, int hbits, char *smem, int32_t *done,
                                         int32_t *abortf) {
    const int tid = threadIdx.x, lane = tid & 63;
    const bool w0 = tid < 64;
    const int64_t s = rp[i], e = rp[i + 1];
    const int len = (int)(e - s);
    const int probe = __builtin_amdgcn_readfirstlane(ilu0_probe);
    const bool pr = probe > 0 && i % probe == 0;
    uint64_t tp[5] = {pr ? (uint64_t)wall_clock64() : 0ull, 0, 0, 0, 0}, t_stage = 0, t_elim = 0, tq = 0;
    // LDS: row values [max_row] | staged values [stage] | row cols [max_row] | staged positions [stage]
    //      | per-pivot staged offsets [max_row + 1] | per-pivot 1/u_rr [max_row] | per-pivot first
    //      upper entry [max_row] | hash keys, positions [2^hbits each]
    // (stage == 0: no staged arrays -- every pivot goes through global memory
    // and reads 1/u_rr there -- so rows of up to ~13.6k entries fit, ilu0_max_row)
    double *rv = reinterpret_cast<double *>(smem);
    double *sv = rv + max_row;
    int32_t *rc = reinterpret_cast<int32_t *>(sv + stage);
    int32_t *sc = rc + max_row;
    int32_t *so = sc + stage;
    double *sd = reinterpret_cast<double *>(((uintptr_t)(so + max_row + 1) + 7) & ~(uintptr_t)7);
    int64_t *su = reinterpret_cast<int64_t *>(sd + max_row);
    int32_t *hk = stage > 0 ? reinterpret_cast<int32_t *>(su + max_row) : so;
    int32_t *hp = hk + (hbits > 0 ? 1 << hbits : 0);
    const uint32_t hmask = (1u << hbits) - 1;
    auto hslot = [&](int32_t c) { return ((uint32_t)c * 2654435761u) >> (32 - hbits); };
    for (int t = tid; t < len; t += ILU0_TPB) {
        rv[t] = lu[s + t];  // (the row's own entries: written by no other row)
        rc[t] = ci[s + t];
    }
    if (hbits > 0) {
        for (int h = tid; h <= (int)hmask; h += ILU0_TPB) hk[h] = -1;
        __syncthreads();
        for (int t = tid; t < len; t += ILU0_TPB) {
            const int32_t c = rc[t];
            uint32_t h = hslot(c);
            while (atomicCAS(&hk[h], -1, c) != -1) h = (h + 1) & hmask;
            hp[h] = t;
        }
    }
    __syncthreads();
    const int dl = (int)(diag[i] - s);
    if (pr) tp[1] = wall_clock64();
    // pivot t's upper part (row rc[t]) goes to so[t] .. so[t + 1] (wave 0 scans)
    if (w0 && stage > 0) {
        int total = 0;
        for (int t0 = 0; t0 < dl; t0 += 64) {
            const int t = t0 + lane;
            int cnt = 0;
            int64_t u0 = 0;
            if (t < dl) {
                const int64_t r = rc[t];
                u0 = diag[r] + 1;
                cnt = (int)(rp[r + 1] - u0);
            }
            int inc = cnt;  // inclusive wave scan
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int v = __shfl_up(inc, o);
                if (lane >= o) inc += v;
            }
            if (t < dl) {
                so[t] = total + inc - cnt;
                su[t] = u0;
            }
            total += __shfl(inc, 63);
        }
        if (lane == 0) so[dl] = total;
    }
    __syncthreads();
    // the staged entries' positions depend on the pattern only: with one segment
    // they are resolved before the wait (DEP), off the dependency chain
    const bool pre = DEP && stage > 0 && so[dl] <= stage;
    if (pre) ilu0_stage_part<DEP, true, false>(0, dl, 0, so[dl], rp, ci, lu, len, hbits, rc, so, su, sc, sv, hk, hp);
    if (pr) tp[2] = wall_clock64();
    if (DEP) {  // every pivot row (an earlier level: already drawn) finished
        if (w0) {
            int ab = 0;
            for (int t0 = 0; t0 < dl && !ab; t0 += 64) {
                const int t = t0 + lane;
                const int32_t k = t < dl ? rc[t] : -1;
                bool ok = k < 0;
                for (int64_t spins = 0;; ++spins) {
                    // (only the flags not yet seen are polled: 64 scattered loads per poll from
                    // ~250 waiting rows measured ~30x slower staging for every row)
                    if (!ok) ok = __hip_atomic_load(done + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                    if (__all(ok)) break;
                    if ((spins & 63) == 63 && __hip_atomic_load(abortf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        ab = 1;
                        break;
                    }
                    if (spins > ILU0_SPIN_MAX) {  // report instead of hanging: every row then stops
                        if (lane == 0) {
                            atomicMax(fail, 3);
                            __hip_atomic_store(abortf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                        ab = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(4);
                }
            }
            if (lane == 0) ilu0_ctl[1] = ab;
        }
        __syncthreads();
        if (ilu0_ctl[1]) return false;
    }
    if (stage > 0)
        for (int t = tid; t < dl; t += ILU0_TPB) sd[t] = ilu0_ld<DEP>(dinv + rc[t]);
    __syncthreads();
    if (pr) tp[3] = wall_clock64();
    int nseg = 0, nglob = 0;
    // pivots in segments [ta, tb) whose upper parts fit the stage together; a
    // pivot whose part alone does not (or no stage) goes through global memory
    for (int ta = 0; ta < dl;) {
        int tb = ta;
        const int base = stage > 0 ? so[ta] : 0;
        if (stage > 0) {  // the last tb with so[tb] - base <= stage
            int hi = dl;
            while (tb < hi) {
                const int m = (tb + hi + 1) >> 1;
                if (so[m] - base <= stage) tb = m; else hi = m - 1;
            }
        }
        if (tb > ta && pre) {
            // DEP, one segment: waves 1-3 stage the values chunk by chunk (CH pivots)
            // while wave 0 eliminates, waiting only for the chunk it needs next
            // (values ~5 us, elimination ~9 us per row: the row's time after its
            // pivots finish is the dependency chain's step)
            if (pr) tq = wall_clock64();
            const int CH = dl > 512 ? (dl + 63) / 64 : 8, nch = (dl + CH - 1) / CH;
            if (tid < 64) ilu0_cnt[tid] = 0;
            __syncthreads();
            if (!w0) {
                for (int cc = 0; cc < nch; ++cc) {
                    const int t0 = cc * CH, t1 = min(dl, t0 + CH);
                    ilu0_stage_part<DEP, false, true>(t0, t1, so[t0], so[t1] - so[t0], rp, ci, lu, len, hbits, rc, so,
                                                      su, sc, sv, hk, hp, so[t0], tid - 64, ILU0_TPB - 64);
                    if (lane == 0) __hip_atomic_fetch_add(ilu0_cnt + cc, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            } else {
                auto wait_chunk = [&](int cc) {
                    for (int64_t spins = 0;
                         __hip_atomic_load(ilu0_cnt + cc, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <
                         ILU0_TPB / 64 - 1;
                         ++spins) {
                        if (spins > ILU0_SPIN_MAX) {  // never expected: report, do not hang
                            if (lane == 0) atomicMax(fail, 3);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                };
                // software pipeline: pivot t computes while pivot t + 1's first entries
                // and pivot t + 2's offsets are in flight; rv[t] and the first update
                // target are read first, so the chain waits for one LDS round trip
                wait_chunk(0);
                int kn = so[0] + lane, en = so[1];
                int lon = kn < en ? sc[kn] : len;
                double vn = kn < en ? sv[kn] : 0.0, dn = sd[0];
                int s2a = dl > 1 ? so[1] : 0, s2b = dl > 1 ? so[2] : 0;  // pivot t + 1's range (next)
                for (int t = 0; t < dl; ++t) {
                    const int lo0 = lon, kc = kn, ec = en;
                    const double v0 = vn, dc = dn;
                    const double pc = rv[t];
                    const double r0 = rv[lo0 < len ? lo0 : t];
                    if (t + 1 < dl) {
                        if ((t + 1) % CH == 0) wait_chunk((t + 1) / CH);
                        kn = s2a + lane;
                        en = s2b;
                        lon = kn < en ? sc[kn] : len;
                        vn = kn < en ? sv[kn] : 0.0;
                        dn = sd[t + 1];
                        s2a = s2b;
                        s2b = t + 3 <= dl ? so[t + 3] : s2b;
                    }
                    if (pc != 0.0) {
                        const double mult = pc * dc;
                        if (lane == 0) rv[t] = mult;
                        if (lo0 < len) rv[lo0] = r0 - mult * v0;
                        for (int kk = kc + 64; kk < ec; kk += 64) {
                            const int lo = sc[kk];
                            if (lo < len) rv[lo] = rv[lo] - mult * sv[kk];
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
            __syncthreads();
            if (pr) t_elim += wall_clock64() - tq;
            ta = tb;
            ++nseg;
            continue;
        }
        if (tb > ta) {
            if (pr) tq = wall_clock64();
            const int cnt = so[tb] - base;
            if (pre)
                ilu0_stage_part<DEP, false, true>(ta, tb, base, cnt, rp, ci, lu, len, hbits, rc, so, su, sc, sv, hk, hp);
            else
                ilu0_stage_part<DEP, true, true>(ta, tb, base, cnt, rp, ci, lu, len, hbits, rc, so, su, sc, sv, hk, hp);
            __syncthreads();
            if (pr) {
                const uint64_t now = wall_clock64();
                t_stage += now - tq;
                tq = now;
            }
            if (w0) {
                // (one wave: its LDS accesses complete in order, so no barrier between pivots;
                // pivot t + 1's first entries and 1/u_rr are read before pivot t's updates --
                // the staged arrays are not written here)
                int k0 = so[ta] - base + lane, e0 = so[ta + 1] - base;
                int lon = k0 < e0 ? sc[k0] : len;
                double vn = k0 < e0 ? sv[k0] : 0.0, dn = sd[ta];
                for (int t = ta; t < tb; ++t) {
                    const int lo0 = lon, kc = k0, ec = e0;
                    const double v0 = vn, dc = dn;
                    if (t + 1 < tb) {
                        k0 = so[t + 1] - base + lane;
                        e0 = so[t + 2] - base;
                        lon = k0 < e0 ? sc[k0] : len;
                        vn = k0 < e0 ? sv[k0] : 0.0;
                        dn = sd[t + 1];
                    }
                    // rv[t] and the first entry the pivot updates are read together (one LDS
                    // round trip per pivot on the chain): positions of pivot t's upper part
                    // are > t and distinct, so nothing writes rv[lo0] in between
                    const double pc = rv[t];
                    const double r0 = rv[lo0 < len ? lo0 : t];
                    if (pc != 0.0) {
                        const double mult = pc * dc;
                        if (lane == 0) rv[t] = mult;
                        if (lo0 < len) rv[lo0] = r0 - mult * v0;
                        for (int kk = kc + 64; kk < ec; kk += 64) {
                            const int lo = sc[kk];
                            if (lo < len) rv[lo] = rv[lo] - mult * sv[kk];
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
            __syncthreads();  // (the next segment overwrites the stage)
            if (pr) t_elim += wall_clock64() - tq;
            ta = tb;
            ++nseg;
            continue;
        }
        const int t = ta++;
        ++nglob;
        if (w0) {
            const double pc = rv[t];
            if (pc != 0.0) {
                const int64_t r = rc[t];
                const double mult = pc * ilu0_ld<DEP>(dinv + r);
                if (lane == 0) rv[t] = mult;
                const int64_t us = diag[r] + 1, ue = rp[r + 1];
                for (int64_t kk = us + lane; kk < ue; kk += 64) {
                    const int32_t j = ci[kk];
                    int lo = len;
                    if (hbits > 0) {  // the column's position in the row (hash)
                        uint32_t h = hslot(j);
                        int32_t key = hk[h];
                        while (key != j && key != -1) {
                            h = (h + 1) & hmask;
                            key = hk[h];
                        }
                        if (key == j) lo = hp[h];
                    } else {  // search j in rc[t+1, len)
                        int a = t + 1, b = len;
                        while (a < b) {
                            const int m = (a + b) >> 1;
                            if (rc[m] < j) a = m + 1; else b = m;
                        }
                        if (a < len && rc[a] == j) lo = a;
                    }
                    if (lo < len) rv[lo] = rv[lo] - mult * ilu0_ld<DEP>(lu + kk);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    __syncthreads();
    if (pr) tp[4] = wall_clock64();
    for (int t = tid; t < len; t += ILU0_TPB) ilu0_st<DEP>(lu + s + t, rv[t]);
    if (tid == 0) {
        const double piv = rv[dl];
        if (piv == 0.0) atomicMax(fail, 2);
        ilu0_st<DEP>(dinv + i, piv == 0.0 ? 0.0 : 1.0 / piv);
    }
    if (DEP) {  // publish: the row's coherent stores complete, then its flag
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (tid == 0) __hip_atomic_store(done + i, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (pr && tid == 0) {
        const uint64_t t5 = wall_clock64();
        printf("[ilu0 row] %ld len %d dl %d staged %d seg %d glob %d | t %lu load %lu wait %lu scan %lu stage %lu "
               "elim %lu rest %lu out %lu\n",
               (long)i, len, dl, stage > 0 ? so[dl] : 0, nseg, nglob, (unsigned long)tp[0],
               (unsigned long)(tp[1] - tp[0]), (unsigned long)(tp[2] - tp[1]), (unsigned long)(tp[3] - tp[2]),
               (unsigned long)t_stage, (unsigned long)t_elim, (unsigned long)(tp[4] - tp[3] - t_stage - t_elim),
               (unsigned long)(t5 - tp[4]));
    }
    return true;
}

__global__ __launch_bounds__(ILU0_TPB) void k_ilu0_level(const int32_t *__restrict__ rows,
                                                         const int64_t *__restrict__ rp,
                                                         const int32_t *__restrict__ ci, double *__restrict__ lu,
                                                         const int64_t *__restrict__ diag, double *__restrict__ dinv,
                                                         int32_t *fail, int max_row, int stage, int hbits) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    (void)ilu0_row<false>(rows[blockIdx.x], rp, ci, lu, diag, dinv, fail, max_row, stage, hbits, smem, nullptr,
                          nullptr);
}

// all levels in one launch: ctr[0] draws rows (rows: level order, so every
// pivot row was drawn earlier -- by a running workgroup -- and the lowest
// unfinished drawn row always has its pivots done: no deadlock); ctr[1] =
// abort flag; done[n] zeroed by the caller
__global__ __launch_bounds__(ILU0_TPB) void k_ilu0_dep(int64_t n, const int32_t *__restrict__ rows,
                                                       const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                       double *lu, const int64_t *__restrict__ diag, double *dinv,
                                                       int32_t *fail, int max_row, int stage, int hbits,
                                                       int32_t *done, int32_t *ctr) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    for (;;) {
        if (threadIdx.x == 0) {
            const int q = atomicAdd(ctr, 1);
            ilu0_ctl[0] = (q >= n || __hip_atomic_load(ctr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ? -1 : q;
        }
        __syncthreads();
        const int q = ilu0_ctl[0];
        __syncthreads();
        if (q < 0) return;
        if (!ilu0_row<true>(rows[q], rp, ci, lu, diag, dinv, fail, max_row, stage, hbits, smem, done, ctr + 1))
            return;
        __syncthreads();
    }
}
#pragma clang fp contract(on)

// the LDS the factorization kernels take for rows of up to max_row entries, `stage` staged
// entries and a 2^hbits-slot column hash
static size_t ilu0_lds_bytes(int64_t max_row, int64_t stage, int hbits) {
    const int64_t m = max_row < 1 ? 1 : max_row;
    // the per-pivot arrays (offsets, 1/u_rr, first entries) exist only with a stage
    const int64_t extra = (stage > 0 ? (m + 1) * 4 + 8 + m * 16 : 0) + (hbits > 0 ? (int64_t)8 << hbits : 0);
    return (size_t)(((m * 12 + stage * 12 + extra) + 15) & ~(int64_t)15);
}
// test knobs (process-wide, pls.ilu0_stage / pls.ilu_dep_grid): a cap on the
// staged entries (0: none staged, every pivot through global memory; small
// values force the segmented path) and on the persistent launch's grid (1: one
// workgroup takes the rows in draw order -- a draw order that is not a
// topological order of the pivot DAG would then stop at the bounded wait)
static int ilu0_stage_cap = -1, ilu0_grid_cap = 0;
void set_ilu0_test_caps(int stage_cap, int grid_cap) {
    ilu0_stage_cap = stage_cap;
    ilu0_grid_cap = grid_cap;
}
// hash slots (at least twice the longest row) and staged entries (the most one
// row needs, at most ILU0_STAGE) that fit the LDS; 0 = none
static void ilu0_plan(int64_t max_row, int64_t max_staged, int &stage, int &hbits) {
    hbits = 7;
    while ((int64_t)1 << hbits < 2 * max_row) ++hbits;
    if (ilu0_lds_bytes(max_row, 0, hbits) > ILU0_LDS) hbits = 0;
    stage = 0;
    int64_t want = std::min<int64_t>(ILU0_STAGE, std::max<int64_t>(256, (max_staged + 63) & ~(int64_t)63));
    if (ilu0_stage_cap >= 0) want = std::min<int64_t>(want, ilu0_stage_cap);
    for (int64_t st = want; st >= std::min<int64_t>(want, 256) && st > 0; st /= 2)
        if (ilu0_lds_bytes(max_row, st, hbits) <= ILU0_LDS) {
            stage = (int)st;
            break;
        }
}
// the longest row with no stage: row values and columns (12 bytes per entry)
int ilu0_max_row() { return (ILU0_LDS - 16) / 12; }
void launch_ilu0_dep(int64_t n, const int32_t *rows, const int64_t *rp, const int32_t *ci, double *lu,
                     const int64_t *diag, double *dinv, int32_t *fail, int64_t max_row, int64_t max_staged,
                     int32_t *done, int32_t *ctr, hipStream_t st) {
    if (n <= 0) return;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)k_ilu0_dep, hipFuncAttributeMaxDynamicSharedMemorySize, ILU0_LDS);
        attr = true;
    }
    int stage = 0, hbits = 0;
    ilu0_plan(max_row, max_staged, stage, hbits);
    const size_t lds = ilu0_lds_bytes(max_row, stage, hbits);
    (void)hipMemsetAsync(done, 0, sizeof(int32_t) * n, st);
    (void)hipMemsetAsync(ctr, 0, sizeof(int32_t) * 2, st);
    // persistent: the workgroups that fit (4 per CU at most), never more than rows
    const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(4, 163840 / (int64_t)(lds + 512)));
    int64_t grid = std::min<int64_t>(n, 256 * per_cu);
    if (ilu0_grid_cap > 0) grid = std::min<int64_t>(grid, ilu0_grid_cap);
    k_ilu0_dep<<<(unsigned)grid, ILU0_TPB, lds, st>>>(n, rows, rp, ci, lu, diag, dinv, fail,
                                                       (int)(max_row < 1 ? 1 : max_row), stage, hbits, done, ctr);
}
void launch_ilu0_level(int64_t nrows_level, const int32_t *rows, const int64_t *rp, const int32_t *ci, double *lu,
                       const int64_t *diag, double *dinv, int32_t *fail, int64_t max_row, int64_t max_staged,
                       hipStream_t st) {
    // caller guarantees max_row <= ilu0_max_row(); LDS sized to the longest row (occupancy for short rows)
    if (nrows_level <= 0) return;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)k_ilu0_level, hipFuncAttributeMaxDynamicSharedMemorySize, ILU0_LDS);
        attr = true;
    }
    int stage = 0, hbits = 0;
    ilu0_plan(max_row, max_staged, stage, hbits);
    k_ilu0_level<<<(unsigned)nrows_level, ILU0_TPB, ilu0_lds_bytes(max_row, stage, hbits), st>>>(
        rows, rp, ci, lu, diag, dinv, fail, (int)(max_row < 1 ? 1 : max_row), stage, hbits);
}

__global__ __launch_bounds__(TPB) void k_lvl_count(int64_t n, const int32_t *order, const int64_t *rp,
                                                   const int64_t *diag, int upper, int64_t *len) {
    const int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (r > n) return;
    if (r == n) { len[n] = 0; return; }
    const int64_t i = order[r];
    len[r] = upper ? (rp[i + 1] - diag[i] - 1) : (diag[i] - rp[i]);
}
__global__ __launch_bounds__(TPB) void k_lvl_fill(int64_t n, const int32_t *order, const int64_t *rp,
                                                  const int32_t *ci, const double *lu, const int64_t *diag, int upper,
                                                  const int64_t *orp, int32_t *oci, double *oval) {
    const int64_t r = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 4;
    const int l = threadIdx.x & 15;
    if (r >= n) return;
    const int64_t i = order[r];
    const int64_t src = upper ? diag[i] + 1 : rp[i];
    const int64_t dst = orp[r], cnt = orp[r + 1] - dst;
    for (int64_t k = l; k < cnt; k += 16) {
        oci[dst + k] = ci[src + k];
        oval[dst + k] = lu[src + k];
    }
}
void launch_lvl_count(int64_t n, const int32_t *order, const int64_t *rp, const int64_t *diag, int upper,
                      int64_t *len, hipStream_t st) {
    k_lvl_count<<<grid_for(n + 1, TPB), TPB, 0, st>>>(n, order, rp, diag, upper, len);
}
void launch_lvl_fill(int64_t n, const int32_t *order, const int64_t *rp, const int32_t *ci, const double *lu,
                     const int64_t *diag, int upper, const int64_t *out_rp, int32_t *out_ci, double *out_val,
                     hipStream_t st) {
    if (n > 0)
        k_lvl_fill<<<grid_for(n * 16, TPB), TPB, 0, st>>>(n, order, rp, ci, lu, diag, upper, out_rp, out_ci,
                                                         out_val);
}

// level of a triangular sweep.  forward (dinv == null): y[i] = b[i] - sum
// backward: y[i] = (y[i] - sum) * dinv[r]
template <int LPR>
__global__ __launch_bounds__(TPB) void k_trsv_level(int64_t r0, int64_t r1, const int32_t *__restrict__ row_of,
                                                    const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                    const double *__restrict__ val, const double *__restrict__ dinv,
                                                    const double *b, double *y) {
    const int sub = threadIdx.x & (LPR - 1);
    const int64_t r = r0 + ((int64_t)blockIdx.x * TPB + threadIdx.x) / LPR;
    if (r >= r1) return;
    const int64_t i = row_of[r];
    const int64_t s = rp[r], e = rp[r + 1];
    double acc = row_dot<LPR, 2, false>(s, e, sub, ci, val, y);
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (sub == 0) {
        if (dinv) y[i] = (y[i] - acc) * dinv[r];
        else y[i] = b[i] - acc;
    }
}

void launch_trsv_level(int64_t r0, int64_t r1, const int32_t *row_of, const int64_t *rp, const int32_t *ci,
                       const double *val, const double *dinv_lvl, const double *b, double *y, int lpr,
                       hipStream_t st) {
    const int64_t rows = r1 - r0;
    if (rows <= 0) return;
    switch (lpr) {
        case 64: k_trsv_level<64><<<grid_for(rows, TPB / 64), TPB, 0, st>>>(r0, r1, row_of, rp, ci, val, dinv_lvl, b, y); break;
        case 32: k_trsv_level<32><<<grid_for(rows, TPB / 32), TPB, 0, st>>>(r0, r1, row_of, rp, ci, val, dinv_lvl, b, y); break;
        case 16: k_trsv_level<16><<<grid_for(rows, TPB / 16), TPB, 0, st>>>(r0, r1, row_of, rp, ci, val, dinv_lvl, b, y); break;
        case 8: k_trsv_level<8><<<grid_for(rows, TPB / 8), TPB, 0, st>>>(r0, r1, row_of, rp, ci, val, dinv_lvl, b, y); break;
        default: k_trsv_level<4><<<grid_for(rows, TPB / 4), TPB, 0, st>>>(r0, r1, row_of, rp, ci, val, dinv_lvl, b, y); break;
    }
}

// Block-Jacobi sweep: one workgroup per diagonal block walks that block's
// levels (rows stored block-major, level-ordered) with only a workgroup
// barrier between levels -- the blocks are independent, so no grid-wide sync
// and no per-level launch.  y is read/written through L1 by the workgroup's
// own waves only (workgroup-scope visibility via __syncthreads()).
template <int LPR>
__global__ __launch_bounds__(512) void k_trsv_blocks(const int64_t *__restrict__ blk_off,
                                                     const int64_t *__restrict__ lvl_ptr,
                                                     const int32_t *__restrict__ row_of,
                                                     const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                     const double *__restrict__ val, const double *__restrict__ dinv,
                                                     const double *b, double *y) {
    const int sub = threadIdx.x & (LPR - 1);
    const int grp = threadIdx.x / LPR;
    constexpr int NG = 512 / LPR;
    const int64_t l0 = blk_off[blockIdx.x], l1 = blk_off[blockIdx.x + 1];
    for (int64_t l = l0; l < l1; ++l) {
        const int64_t rs = lvl_ptr[l], re = lvl_ptr[l + 1];
        for (int64_t r = rs + grp; r < re; r += NG) {
            const int64_t i = row_of[r];
            const int64_t s = rp[r], e = rp[r + 1];
            double acc = row_dot<LPR, 2, false>(s, e, sub, ci, val, y);
#pragma unroll
            for (int o = LPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
            if (sub == 0) {
                if (dinv) y[i] = (y[i] - acc) * dinv[r];
                else y[i] = b[i] - acc;
            }
        }
        __syncthreads();
    }
}

void launch_trsv_blocks(int64_t nblocks, const int64_t *blk_off, const int64_t *lvl_ptr, const int32_t *row_of,
                        const int64_t *rp, const int32_t *ci, const double *val, const double *dinv_lvl,
                        const double *b, double *y, int lpr, hipStream_t st) {
    if (nblocks <= 0) return;
    switch (lpr) {
        case 64: k_trsv_blocks<64><<<(unsigned)nblocks, 512, 0, st>>>(blk_off, lvl_ptr, row_of, rp, ci, val, dinv_lvl, b, y); break;
        case 32: k_trsv_blocks<32><<<(unsigned)nblocks, 512, 0, st>>>(blk_off, lvl_ptr, row_of, rp, ci, val, dinv_lvl, b, y); break;
        case 16: k_trsv_blocks<16><<<(unsigned)nblocks, 512, 0, st>>>(blk_off, lvl_ptr, row_of, rp, ci, val, dinv_lvl, b, y); break;
        case 8: k_trsv_blocks<8><<<(unsigned)nblocks, 512, 0, st>>>(blk_off, lvl_ptr, row_of, rp, ci, val, dinv_lvl, b, y); break;
        default: k_trsv_blocks<4><<<(unsigned)nblocks, 512, 0, st>>>(blk_off, lvl_ptr, row_of, rp, ci, val, dinv_lvl, b, y); break;
    }
}

// ============================================================== SELL-64 ====
// Sliced ELLPACK, slice height = one 64-lane wave: slice s holds rows
// [64 s, 64 s + 64), entry k of its rows stored contiguously
// (sptr[s] + 64 k + lane).  Lane = row, so the val / col streams are fully
// coalesced, no cross-lane reduction is needed, each row sums its entries in
// column order, and for banded / stencil columns the 64 x gathers of one
// wave-instruction hit 4-5 consecutive cache lines instead of 64.
__global__ __launch_bounds__(TPB) void k_sell_slice_len(int64_t nrows, int64_t nslices, const int64_t *rp,
                                                        int64_t *slen) {
    const int64_t sl = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (sl > nslices) return;
    if (sl == nslices) { if (lane == 0) slen[nslices] = 0; return; }
    const int64_t row = sl * 64 + lane;
    int64_t len = row < nrows ? rp[row + 1] - rp[row] : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t t = __shfl_xor(len, o);
        len = t > len ? t : len;
    }
    if (lane == 0) slen[sl] = 64 * len;
}

__global__ __launch_bounds__(TPB) void k_sell_fill(int64_t nrows, int64_t nslices, const int64_t *rp, const int32_t *ci,
                                                   const double *val, const int64_t *sptr, int32_t *scol, double *sval) {
    const int64_t sl = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (sl >= nslices) return;
    const int64_t row = sl * 64 + lane;
    const int64_t base = sptr[sl];
    const int64_t L = (sptr[sl + 1] - base) >> 6;
    const int64_t s0 = row < nrows ? rp[row] : 0;
    const int64_t len = row < nrows ? rp[row + 1] - s0 : 0;
    const int32_t padc = len > 0 ? ci[s0 + len - 1] : 0;
    for (int64_t k = 0; k < L; ++k) {
        const int64_t pos = base + k * 64 + lane;
        if (k < len) {
            scol[pos] = ci[s0 + k];
            sval[pos] = val[s0 + k];
        } else {
            scol[pos] = padc;
            sval[pos] = 0.0;
        }
    }
}

// TAG only separates the outer-operator instantiation (TAG 1: y = A x of the
// Krylov loop) from the preconditioner's block products in profiles.
template <int U, int TAG, bool HALO>
__global__ __launch_bounds__(TPB) void k_sell_spmv(int64_t nrows, int64_t nslices, const int64_t *__restrict__ sptr,
                                                   const int32_t *__restrict__ scol, const double *__restrict__ sval,
                                                   const double *__restrict__ x, double *__restrict__ y, double alpha,
                                                   double beta, const double *__restrict__ z,
                                                   const double *__restrict__ ghost, int32_t nlocal) {
    const int lane = threadIdx.x & 63;
    const int64_t sl = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (TPB / 64) + (threadIdx.x >> 6)));
    if (sl >= nslices) return;
    const int64_t base = sptr[sl];
    const int64_t L = (sptr[sl + 1] - base) >> 6;
    const int32_t *cp = scol + base + lane;
    const double *vp = sval + base + lane;
    double acc = 0.0;
    for (int64_t k0 = 0; k0 < L; k0 += U) {
        int32_t c[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t k = k0 + u;
            const int64_t kk = k < L ? k : L - 1;  // wave-uniform clamp, value masked
            c[u] = __builtin_nontemporal_load(cp + kk * 64);
            const double t = __builtin_nontemporal_load(vp + kk * 64);
            v[u] = k < L ? t : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (HALO) {
                const bool loc = c[u] < nlocal;
                const double xv = loc ? x[(uint32_t)c[u]] : ghost[(uint32_t)(c[u] - nlocal)];
                acc += v[u] * xv;
            } else {
                acc += v[u] * x[(uint32_t)c[u]];
            }
        }
    }
    const int64_t row = sl * 64 + lane;
    if (row < nrows) {
        double r = alpha * acc;
        if (beta != 0.0) r += beta * z[row];
        y[row] = r;
    }
}

int64_t sell_nslices(int64_t nrows) { return (nrows + 63) / 64; }

void launch_sell_slice_len(int64_t nrows, const int64_t *rp, int64_t *slen, hipStream_t st) {
    const int64_t ns = sell_nslices(nrows);
    k_sell_slice_len<<<grid_for((ns + 1) * 64, TPB), TPB, 0, st>>>(nrows, ns, rp, slen);
}
void launch_sell_fill(int64_t nrows, const int64_t *rp, const int32_t *ci, const double *val, const int64_t *sptr,
                      int32_t *scol, double *sval, hipStream_t st) {
    const int64_t ns = sell_nslices(nrows);
    if (ns > 0) k_sell_fill<<<grid_for(ns * 64, TPB), TPB, 0, st>>>(nrows, ns, rp, ci, val, sptr, scol, sval);
}
void launch_sell_spmv(int64_t nrows, const int64_t *sptr, const int32_t *scol, const double *sval, const double *x,
                      double *y, double alpha, double beta, const double *z, int tag, const double *ghost,
                      int64_t nlocal, hipStream_t st) {
    const int64_t ns = sell_nslices(nrows);
    if (ns <= 0) return;
    const unsigned g = grid_for(ns, TPB / 64);
    const int32_t nl = (int32_t)nlocal;
    if (ghost) {
        if (tag) k_sell_spmv<8, 1, true><<<g, TPB, 0, st>>>(nrows, ns, sptr, scol, sval, x, y, alpha, beta, z, ghost, nl);
        else k_sell_spmv<8, 0, true><<<g, TPB, 0, st>>>(nrows, ns, sptr, scol, sval, x, y, alpha, beta, z, ghost, nl);
    } else {
        if (tag) k_sell_spmv<8, 1, false><<<g, TPB, 0, st>>>(nrows, ns, sptr, scol, sval, x, y, alpha, beta, z, ghost, nl);
        else k_sell_spmv<8, 0, false><<<g, TPB, 0, st>>>(nrows, ns, sptr, scol, sval, x, y, alpha, beta, z, ghost, nl);
    }
}

// ====================================================== SELL-64 / D16 =====
// Compressed SELL-64: entry k of a lane's stream stores a 16-bit column delta
// (col_k - col_{k-1}, 1..65535) instead of an int32 column, 10 B per entry
// instead of 12.  A delta of 0 means "start the next segment": the column is
// the next of the lane's D16_SEG absolute segment bases (the first entry, and
// every jump > 65535 -- field-block changes, ghost columns).  Padding entries
// are segment starts with value 0.0 (the base index clamps to the last one).
// Lanes per row: a slice is 64 lanes; LPR = 1 (64 rows, lane = row) for rows
// whose neighbours use neighbouring columns, LPR = 8 (8 rows, entry j of a row
// on lane j % 8) for "wide" rows whose neighbours' columns lie far apart (a
// pressure row couples to runs of ~(n_u / n_p) displacement columns): there a
// lane-per-row gather touches 64 cache lines per instruction, 8 lanes per row
// read 8 consecutive columns.  The LPR partial sums are combined by lane
// shuffles (LPR = 1 rows sum in CSR order: bitwise equal to SELL-64).
// Layout for 16-B-per-lane loads (1 KiB per wave instruction):
//   deltas  dl[base + (k / 8) * 512 + lane * 8 + k % 8]   (one uint4 = 8 deltas)
//   values  dv[base + (k / 2) * 128 + lane * 2 + k % 2]   (one double2 = 2 values)
//   bases   seg[(slice * 64 + lane) * D16_SEG + j]        (one int4 per lane)
//   slices  sfirst[slice] (first row), slpr[slice] (lanes per row)
__device__ __forceinline__ void d16_lane(int64_t sl, int lane, const int64_t *sfirst, const int32_t *slpr,
                                         int64_t nrows, int64_t &row, int &lpr, int &sub,
                                         const int32_t *rowmap) {
    lpr = slpr[sl];
    row = sfirst[sl] + lane / lpr;
    sub = lane % lpr;
    if (row >= sfirst[sl + 1] || row >= nrows) row = -1;
    else if (rowmap) row = rowmap[row];
}

__global__ __launch_bounds__(TPB) void k_d16_slice_len(int64_t nslices, const int64_t *sfirst, const int32_t *slpr,
                                                       const int64_t *rp, int64_t nrows, int64_t *slen,
                                                       const int32_t *rowmap) {
    const int64_t sl = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (sl > nslices) return;
    if (sl == nslices) { if (lane == 0) slen[nslices] = 0; return; }
    int64_t row;
    int lpr, sub;
    d16_lane(sl, lane, sfirst, slpr, nrows, row, lpr, sub, rowmap);
    const int64_t len = row >= 0 ? rp[row + 1] - rp[row] : 0;
    int64_t mine = len > sub ? (len - sub + lpr - 1) / lpr : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t t = __shfl_xor(mine, o);
        mine = t > mine ? t : mine;
    }
    if (lane == 0) slen[sl] = 64 * ((mine + 7) & ~(int64_t)7);
}

// segments each lane's entry stream needs; *maxseg = max over lanes
__global__ __launch_bounds__(TPB) void k_d16_count(int64_t nslices, const int64_t *sfirst, const int32_t *slpr,
                                                   const int64_t *rp, const int32_t *ci, int64_t nrows,
                                                   int32_t *maxseg, const int32_t *rowmap) {
    const int64_t sl = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (sl >= nslices) return;
    int64_t row;
    int lpr, sub;
    d16_lane(sl, lane, sfirst, slpr, nrows, row, lpr, sub, rowmap);
    if (row < 0) return;
    const int64_t s = rp[row], e = rp[row + 1];
    int nseg = 0;
    int64_t last = -1;
    for (int64_t k = s + sub; k < e; k += lpr) {
        const int64_t c = ci[k];
        if (last < 0 || c - last > 65535 || c <= last) ++nseg;
        last = c;
    }
    if (nseg > 0) atomicMax(maxseg, nseg);
}

__global__ __launch_bounds__(TPB) void k_d16_fill(int64_t nslices, const int64_t *sfirst, const int32_t *slpr,
                                                  const int64_t *rp, const int32_t *ci, const double *val,
                                                  int64_t nrows, const int64_t *sptr, uint16_t *dl, double *dv,
                                                  int32_t *seg, int nsegs, const int32_t *rowmap) {
    const int64_t sl = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (sl >= nslices) return;
    int64_t row;
    int lpr, sub;
    d16_lane(sl, lane, sfirst, slpr, nrows, row, lpr, sub, rowmap);
    const int64_t base = sptr[sl];
    const int64_t L = (sptr[sl + 1] - base) >> 6;
    const int64_t s0 = row >= 0 ? rp[row] : 0;
    const int64_t len = row >= 0 ? rp[row + 1] - s0 : 0;
    const int64_t slot = sl * 64 + lane;
    int nseg = 0;
    int32_t last = 0;
    for (int64_t k = 0; k < L; ++k) {
        const int64_t j = k * lpr + sub;  // this lane's k-th entry of the row
        uint16_t d = 0;
        double v = 0.0;
        if (j < len) {
            const int32_t c = ci[s0 + j];
            v = val[s0 + j];
            const int64_t gap = (int64_t)c - (int64_t)last;
            if (k == 0 || gap > 65535 || gap <= 0) {
                seg[slot * nsegs + nseg++] = c;
            } else {
                d = (uint16_t)gap;
            }
            last = c;
        }
        dl[base + (k >> 3) * 512 + lane * 8 + (k & 7)] = d;
        dv[base + (k >> 1) * 128 + lane * 2 + (k & 1)] = v;
    }
    if (nseg == 0) seg[slot * nsegs + nseg++] = 0;
    for (int j = nseg; j < nsegs; ++j) seg[slot * nsegs + j] = seg[slot * nsegs + nseg - 1];
}

// first column of every row (-1: empty row) -- input of the host slice plan
__global__ __launch_bounds__(TPB) void k_first_col(int64_t nrows, const int64_t *rp, const int32_t *ci, int32_t *c0) {
    const int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (r < nrows) c0[r] = rp[r + 1] > rp[r] ? ci[rp[r]] : -1;
}

typedef int32_t d16_i4 __attribute__((ext_vector_type(4)));
typedef uint32_t d16_u4 __attribute__((ext_vector_type(4)));
typedef double d16_d2 __attribute__((ext_vector_type(2)));

__constant__ int d16_xcd_map;  // set once by launch_d16_spmv (pls.d16_xcd)

template <int G2, int TAG, bool HALO, int SEG>
__global__ __launch_bounds__(TPB) void k_d16_spmv(int64_t nrows, int64_t nslices, const int64_t *__restrict__ sptr,
                                                  const int64_t *__restrict__ sfirst,
                                                  const int32_t *__restrict__ slpr,
                                                  const uint16_t *__restrict__ dl, const double *__restrict__ dv,
                                                  const int32_t *__restrict__ seg, const double *__restrict__ x,
                                                  double *__restrict__ y, double alpha, double beta,
                                                  const double *__restrict__ z, const double *__restrict__ ghost,
                                                  int32_t nlocal, const int32_t *__restrict__ slist,
                                                  const int32_t *__restrict__ rowmap) {
    static_assert(SEG == 4 || SEG == 8, "segment bases are one or two int4 per lane");
    const int lane = threadIdx.x & 63;
    // nslices: slices this launch processes -- all of them, or the subset
    // listed in slist (interior / halo rows of a distributed product)
    // d16_xcd_map (pls.d16_xcd 1): workgroup b runs on XCD b % 8; give each XCD a
    // contiguous range of slices (its L2 then holds one window of x) instead
    // of every 8th slice
    unsigned blk = blockIdx.x;
    if (d16_xcd_map) {
        const unsigned per = (gridDim.x + 7) / 8;
        blk = (blockIdx.x % 8) * per + blockIdx.x / 8;
    }
    const int64_t idx = __builtin_amdgcn_readfirstlane((int)(blk * (TPB / 64) + (threadIdx.x >> 6)));
    if (idx >= nslices) return;
    const int64_t sl = slist ? (int64_t)__builtin_amdgcn_readfirstlane(slist[idx]) : idx;
    const int64_t base = sptr[sl];
    const int64_t L = (sptr[sl + 1] - base) >> 6;  // multiple of 8
    const int lpr = slpr[sl];
    const int64_t r0 = sfirst[sl], r1 = sfirst[sl + 1];
    const int64_t row = r0 + lane / lpr;
    const d16_i4 sb = __builtin_nontemporal_load(reinterpret_cast<const d16_i4 *>(seg) + (sl * 64 + lane) * (SEG / 4));
    d16_i4 sb2 = sb;
    if (SEG == 8) sb2 = __builtin_nontemporal_load(reinterpret_cast<const d16_i4 *>(seg) + (sl * 64 + lane) * 2 + 1);
    const d16_u4 *dp = reinterpret_cast<const d16_u4 *>(dl + base) + lane;
    const d16_d2 *vp = reinterpret_cast<const d16_d2 *>(dv + base) + lane;
    int32_t col = 0;
    int si = 0;
    double acc = 0.0;
    const int64_t ng = L >> 3;
    for (int64_t g0 = 0; g0 < ng; g0 += G2) {
        d16_u4 d[G2];
        d16_d2 v[G2][4];
#pragma unroll
        for (int u = 0; u < G2; ++u) {
            const int64_t g = g0 + u < ng ? g0 + u : ng - 1;  // wave-uniform clamp, values masked
            d[u] = __builtin_nontemporal_load(dp + g * 64);
#pragma unroll
            for (int q = 0; q < 4; ++q) v[u][q] = __builtin_nontemporal_load(vp + (g * 4 + q) * 64);
        }
#pragma unroll
        for (int u = 0; u < G2; ++u) {
            if (g0 + u >= ng) break;
            const uint32_t w[4] = {d[u].x, d[u].y, d[u].z, d[u].w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int32_t dd = (int32_t)((w[e >> 1] >> ((e & 1) * 16)) & 0xffffu);
                int32_t b = si == 0 ? sb.x : si == 1 ? sb.y : si == 2 ? sb.z : sb.w;
                if (SEG == 8 && si >= 4) b = si == 4 ? sb2.x : si == 5 ? sb2.y : si == 6 ? sb2.z : sb2.w;
                col = dd == 0 ? b : col + dd;
                si += dd == 0 ? 1 : 0;
                const double a = (e & 1) ? v[u][e >> 1].y : v[u][e >> 1].x;
                if (HALO) {
                    const bool loc = col < nlocal;
                    const double xv = loc ? x[(uint32_t)col] : ghost[(uint32_t)(col - nlocal)];
                    acc += a * xv;
                } else {
                    acc += a * x[(uint32_t)col];
                }
            }
        }
    }
    if (lpr > 1) {  // wave-uniform: combine the LPR partial sums of a row
        for (int o = 1; o < lpr; o <<= 1) acc += __shfl_xor(acc, o);
        if (lane % lpr) return;
    }
    if (row < r1) {
        // rowmap: slices hold rows sorted by length inside windows (SELL-C-sigma);
        // the lane's result goes to its row's place
        const int64_t yr = rowmap ? (int64_t)rowmap[row] : row;
        double r = alpha * acc;
        if (beta != 0.0) r += beta * z[yr];
        y[yr] = r;
    }
}

void launch_d16_slice_len(int64_t nslices, const int64_t *sfirst, const int32_t *slpr, const int64_t *rp,
                          int64_t nrows, int64_t *slen, hipStream_t st, const int32_t *rowmap) {
    k_d16_slice_len<<<grid_for((nslices + 1) * 64, TPB), TPB, 0, st>>>(nslices, sfirst, slpr, rp, nrows, slen, rowmap);
}
void launch_d16_count(int64_t nslices, const int64_t *sfirst, const int32_t *slpr, const int64_t *rp,
                      const int32_t *ci, int64_t nrows, int32_t *maxseg, hipStream_t st, const int32_t *rowmap) {
    if (nslices > 0)
        k_d16_count<<<grid_for(nslices * 64, TPB), TPB, 0, st>>>(nslices, sfirst, slpr, rp, ci, nrows, maxseg, rowmap);
}
void launch_d16_fill(int64_t nslices, const int64_t *sfirst, const int32_t *slpr, const int64_t *rp,
                     const int32_t *ci, const double *val, int64_t nrows, const int64_t *sptr, uint16_t *dl,
                     double *dv, int32_t *seg, int nsegs, hipStream_t st, const int32_t *rowmap) {
    if (nslices > 0)
        k_d16_fill<<<grid_for(nslices * 64, TPB), TPB, 0, st>>>(nslices, sfirst, slpr, rp, ci, val, nrows, sptr, dl,
                                                                dv, seg, nsegs, rowmap);
}
void launch_first_col(int64_t nrows, const int64_t *rp, const int32_t *ci, int32_t *c0, hipStream_t st) {
    if (nrows > 0) k_first_col<<<grid_for(nrows, TPB), TPB, 0, st>>>(nrows, rp, ci, c0);
}
template <int G2, int SEG>
static void d16_dispatch(unsigned g, hipStream_t st, int64_t nrows, int64_t ns, const int64_t *sptr,
                         const int64_t *sfirst, const int32_t *slpr, const uint16_t *dl, const double *dv,
                         const int32_t *seg, const double *x, double *y, double alpha, double beta, const double *z,
                         int tag, const double *ghost, int32_t nl, const int32_t *slist, const int32_t *rm, size_t shm) {
    if (ghost) {
        if (tag) k_d16_spmv<G2, 1, true, SEG><<<g, TPB, shm, st>>>(nrows, ns, sptr, sfirst, slpr, dl, dv, seg, x, y, alpha, beta, z, ghost, nl, slist, rm);
        else k_d16_spmv<G2, 0, true, SEG><<<g, TPB, shm, st>>>(nrows, ns, sptr, sfirst, slpr, dl, dv, seg, x, y, alpha, beta, z, ghost, nl, slist, rm);
    } else {
        if (tag) k_d16_spmv<G2, 1, false, SEG><<<g, TPB, shm, st>>>(nrows, ns, sptr, sfirst, slpr, dl, dv, seg, x, y, alpha, beta, z, ghost, nl, slist, rm);
        else k_d16_spmv<G2, 0, false, SEG><<<g, TPB, shm, st>>>(nrows, ns, sptr, sfirst, slpr, dl, dv, seg, x, y, alpha, beta, z, ghost, nl, slist, rm);
    }
}
template <int SEG>
static void d16_unrolled(int unroll, unsigned g, hipStream_t st, int64_t nrows, int64_t nslices, const int64_t *sptr,
                         const int64_t *sfirst, const int32_t *slpr, const uint16_t *dl, const double *dv,
                         const int32_t *seg, const double *x, double *y, double alpha, double beta, const double *z,
                         int tag, const double *ghost, int32_t nl, const int32_t *slist, const int32_t *rm, size_t shm) {
    switch (unroll) {
        case 1: d16_dispatch<1, SEG>(g, st, nrows, nslices, sptr, sfirst, slpr, dl, dv, seg, x, y, alpha, beta, z, tag, ghost, nl, slist, rm, shm); break;
        case 2: d16_dispatch<2, SEG>(g, st, nrows, nslices, sptr, sfirst, slpr, dl, dv, seg, x, y, alpha, beta, z, tag, ghost, nl, slist, rm, shm); break;
        default: d16_dispatch<4, SEG>(g, st, nrows, nslices, sptr, sfirst, slpr, dl, dv, seg, x, y, alpha, beta, z, tag, ghost, nl, slist, rm, shm); break;
    }
}
static int d16_xcd_host = 0;
void set_d16_xcd(int on) {
    if (on == d16_xcd_host) return;
    d16_xcd_host = on;
    if (hipMemcpyToSymbol(HIP_SYMBOL(d16_xcd_map), &on, sizeof(int)) != hipSuccess) d16_xcd_host = 0;
}
void launch_d16_spmv(int64_t nrows, int64_t nslices, const int64_t *sptr, const int64_t *sfirst, const int32_t *slpr,
                     const uint16_t *dl, const double *dv, const int32_t *seg, int nsegs, const double *x, double *y,
                     double alpha, double beta, const double *z, int tag, const double *ghost, int64_t nlocal,
                     int unroll, hipStream_t st, const int32_t *slist, const int32_t *rowmap, size_t lds_reserve) {
    if (nslices <= 0) return;
    unsigned g = grid_for(nslices, TPB / 64);
    if (d16_xcd_host) g = (g + 7) / 8 * 8;  // every XCD range the same length (surplus blocks exit)
    const int32_t nl = (int32_t)nlocal;
    if (nsegs == 8) d16_unrolled<8>(unroll, g, st, nrows, nslices, sptr, sfirst, slpr, dl, dv, seg, x, y, alpha, beta, z, tag, ghost, nl, slist, rowmap, lds_reserve);
    else d16_unrolled<4>(unroll, g, st, nrows, nslices, sptr, sfirst, slpr, dl, dv, seg, x, y, alpha, beta, z, tag, ghost, nl, slist, rowmap, lds_reserve);
}

// ============================================================ SELL/B3 ======
// Row triples of FE vector fields: the 3 components of a P2 node have the same
// sparsity pattern, so a triple shares one column list.  B3_LPT lanes per
// triple (entry j of the triple's list on lane j % B3_LPT), slices of 64 /
// B3_LPT triples (sorted by length inside windows, tmap[position] = the
// triple's first row); per lane entry kk one column (one x gather serves 3
// rows) and 3 values:  col[base + kk * 64 + lane],
// val[3 * base + (3 kk + r) * 64 + lane].  The lanes' partial sums of a row
// combine by DPP (quad_perm xor 1, xor 2).
constexpr int B3_LPT = 4;

// flag[r] = 1 when rows r, r + 1, r + 2 have the same column list
__global__ __launch_bounds__(TPB) void k_triple_flags(int64_t n, const int64_t *rp, const int32_t *ci, uint8_t *flag) {
    const int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (r >= n) return;
    uint8_t f = 0;
    if (r + 2 < n) {
        const int64_t s0 = rp[r], len = rp[r + 1] - s0;
        if (len > 0 && rp[r + 2] - rp[r + 1] == len && rp[r + 3] - rp[r + 2] == len) {
            const int64_t s1 = rp[r + 1], s2 = rp[r + 2];
            f = 1;
            for (int64_t k = 0; k < len && f; ++k) f = (ci[s0 + k] == ci[s1 + k] && ci[s0 + k] == ci[s2 + k]) ? 1 : 0;
        }
    }
    flag[r] = f;
}
void launch_triple_flags(int64_t n, const int64_t *rp, const int32_t *ci, uint8_t *flag, hipStream_t st) {
    if (n > 0) k_triple_flags<<<grid_for(n, TPB), TPB, 0, st>>>(n, rp, ci, flag);
}
int b3_lanes_per_triple() { return B3_LPT; }

__global__ __launch_bounds__(TPB) void k_b3_fill(int64_t nslices, int64_t ntrip, const int64_t *bptr,
                                                 const int32_t *tmap, const int64_t *rp, const int32_t *ci,
                                                 const double *val, int32_t *bcol, double *bval) {
    const int64_t sl = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63, sub = lane % B3_LPT;
    if (sl >= nslices) return;
    const int64_t base = bptr[sl], L = (bptr[sl + 1] - base) >> 6;
    const int64_t pos = sl * (64 / B3_LPT) + lane / B3_LPT;
    const int64_t h = pos < ntrip ? tmap[pos] : -1;
    const int64_t s0 = h >= 0 ? rp[h] : 0, len = h >= 0 ? rp[h + 1] - s0 : 0;
    const int32_t c0 = len > 0 ? ci[s0] : 0;
    for (int64_t kk = 0; kk < L; ++kk) {
        const int64_t k = kk * B3_LPT + sub;
        const bool in = k < len;
        bcol[base + kk * 64 + lane] = in ? ci[s0 + k] : c0;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int64_t sj = h >= 0 ? rp[h + j] : 0;
            bval[3 * base + (3 * kk + j) * 64 + lane] = in ? val[sj + k] : 0.0;
        }
    }
}

void launch_b3_fill(int64_t nslices, int64_t ntrip, const int64_t *bptr, const int32_t *tmap, const int64_t *rp,
                    const int32_t *ci, const double *val, int32_t *bcol, double *bval, hipStream_t st) {
    if (nslices > 0)
        k_b3_fill<<<grid_for(nslices * 64, TPB), TPB, 0, st>>>(nslices, ntrip, bptr, tmap, rp, ci, val, bcol, bval);
}

__device__ __forceinline__ double b3_dpp(double v, int ctrl_xor) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    if (ctrl_xor == 1)
        return __hiloint2double(__builtin_amdgcn_update_dpp(0, hi, 0xB1, 0xF, 0xF, false),
                                __builtin_amdgcn_update_dpp(0, lo, 0xB1, 0xF, 0xF, false));
    return __hiloint2double(__builtin_amdgcn_update_dpp(0, hi, 0x4E, 0xF, 0xF, false),
                            __builtin_amdgcn_update_dpp(0, lo, 0x4E, 0xF, 0xF, false));
}

template <int TAG>
__global__ __launch_bounds__(TPB) void k_b3_spmv(int64_t nslices, int64_t ntrip, const int64_t *__restrict__ bptr,
                                                 const int32_t *__restrict__ tmap, const int32_t *__restrict__ bcol,
                                                 const double *__restrict__ bval, const double *__restrict__ x,
                                                 double *__restrict__ y, double alpha, double beta,
                                                 const double *__restrict__ z) {
    const int64_t sl = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (TPB / 64) + (threadIdx.x >> 6)));
    if (sl >= nslices) return;
    const int lane = threadIdx.x & 63;
    const int64_t base = bptr[sl], L = (bptr[sl + 1] - base) >> 6;
    const int32_t *cp = bcol + base + lane;
    const double *vp = bval + 3 * base + lane;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    int64_t k = 0;
    for (; k + 4 <= L; k += 4) {  // 4 entries per lane in flight
        int32_t c[4];
        double v[4][3], xv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) c[u] = __builtin_nontemporal_load(cp + (k + u) * 64);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
            for (int j = 0; j < 3; ++j) v[u][j] = __builtin_nontemporal_load(vp + (3 * (k + u) + j) * 64);
            xv[u] = x[(uint32_t)c[u]];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a0 += v[u][0] * xv[u];
            a1 += v[u][1] * xv[u];
            a2 += v[u][2] * xv[u];
        }
    }
    for (; k < L; ++k) {
        const double xv = x[(uint32_t)cp[k * 64]];
        a0 += vp[(3 * k) * 64] * xv;
        a1 += vp[(3 * k + 1) * 64] * xv;
        a2 += vp[(3 * k + 2) * 64] * xv;
    }
    static_assert(B3_LPT == 4, "two DPP steps combine the lanes of a triple");
    a0 += b3_dpp(a0, 1); a1 += b3_dpp(a1, 1); a2 += b3_dpp(a2, 1);
    a0 += b3_dpp(a0, 2); a1 += b3_dpp(a1, 2); a2 += b3_dpp(a2, 2);
    const int64_t pos = sl * (64 / B3_LPT) + lane / B3_LPT;
    if (pos >= ntrip || (lane % B3_LPT) >= 3) return;
    // lanes 0, 1, 2 of a triple write its rows 0, 1, 2
    const int j = lane % B3_LPT;
    const int64_t row = tmap[pos] + j;
    const double acc = j == 0 ? a0 : j == 1 ? a1 : a2;
    double r = alpha * acc;
    if (beta != 0.0) r += beta * z[row];
    y[row] = r;
}
void launch_b3_spmv(int64_t nslices, int64_t ntrip, const int64_t *bptr, const int32_t *tmap, const int32_t *bcol,
                    const double *bval, const double *x, double *y, double alpha, double beta, const double *z,
                    int tag, hipStream_t st) {
    if (nslices <= 0) return;
    const unsigned g = grid_for(nslices, TPB / 64);
    if (tag) k_b3_spmv<1><<<g, TPB, 0, st>>>(nslices, ntrip, bptr, tmap, bcol, bval, x, y, alpha, beta, z);
    else k_b3_spmv<0><<<g, TPB, 0, st>>>(nslices, ntrip, bptr, tmap, bcol, bval, x, y, alpha, beta, z);
}

// rows whose last (largest) column is a ghost column (rows sorted): flag 1
__global__ __launch_bounds__(TPB) void k_row_has_ghost(int64_t nrows, const int64_t *rp, const int32_t *ci,
                                                       int64_t nlocal, uint8_t *flag) {
    const int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (r < nrows) flag[r] = (rp[r + 1] > rp[r] && ci[rp[r + 1] - 1] >= nlocal) ? 1 : 0;
}
void launch_row_has_ghost(int64_t nrows, const int64_t *rp, const int32_t *ci, int64_t nlocal, uint8_t *flag,
                          hipStream_t st) {
    if (nrows > 0) k_row_has_ghost<<<grid_for(nrows, TPB), TPB, 0, st>>>(nrows, rp, ci, nlocal, flag);
}

// ================================================= level-aligned SELL-64 ====
// Triangular factors for the sweeps: rows grouped by (block, level), every
// group padded to whole 64-row slices, entry k of a slice's rows contiguous
// (sptr[s] + 64 k + lane).  Lane = row: coalesced val/col loads, no lane
// reduction, and the U entries a lane keeps in flight are independent of the
// level barrier.  Padding entries are discarded by a select (never multiplied
// into the sum), so uninitialised y entries cannot leak NaNs.
__global__ __launch_bounds__(TPB) void k_tri_fill(int64_t nslices, const int32_t *slot_row, const int32_t *slot_len,
                                                  const int64_t *rp, const int32_t *ci, const double *lu,
                                                  const int64_t *diag, const double *dinv, int upper,
                                                  const int64_t *sptr, int32_t *ocol, double *oval, double *odinv) {
    const int64_t sl = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (sl >= nslices) return;
    const int64_t slot = sl * 64 + lane;
    const int32_t i = slot_row[slot];
    const int32_t len = slot_len[slot];
    const int64_t base = sptr[sl];
    const int64_t L = (sptr[sl + 1] - base) >> 6;
    const int64_t src = (i < 0) ? 0 : (upper ? diag[i] + 1 : rp[i]);
    for (int64_t k = 0; k < L; ++k) {
        const int64_t pos = base + k * 64 + lane;
        if (k < len) {
            ocol[pos] = ci[src + k];
            oval[pos] = lu[src + k];
        } else {
            ocol[pos] = 0;
            oval[pos] = 0.0;
        }
    }
    if (odinv) odinv[slot] = (i < 0) ? 1.0 : dinv[i];
}

template <int U>
__device__ __forceinline__ void tri_slice(int64_t sl, int lane, const int64_t *__restrict__ sptr,
                                          const int32_t *__restrict__ slot_row, const int32_t *__restrict__ slot_len,
                                          const int32_t *__restrict__ col, const double *__restrict__ val,
                                          const double *__restrict__ sdinv, const double *b, double *y) {
    const int64_t slot = sl * 64 + lane;
    const int32_t i = slot_row[slot];
    const int32_t len = slot_len[slot];
    const int64_t base = sptr[sl];
    const int64_t L = (sptr[sl + 1] - base) >> 6;
    const int32_t *cp = col + base + lane;
    const double *vp = val + base + lane;
    double acc = 0.0;
    for (int64_t k0 = 0; k0 < L; k0 += U) {
        int32_t c[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t kk = (k0 + u < L) ? k0 + u : L - 1;
            c[u] = cp[kk * 64];
            v[u] = vp[kk * 64];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double t = v[u] * y[(uint32_t)c[u]];
            acc += (k0 + u < len) ? t : 0.0;
        }
    }
    if (i >= 0) {
        if (sdinv) y[i] = (y[i] - acc) * sdinv[slot];
        else y[i] = b[i] - acc;
    }
}

// one workgroup per block: goff[blk]..goff[blk+1] groups, gslice[g] slices
__global__ __launch_bounds__(1024) void k_tri_blocks(const int64_t *__restrict__ goff,
                                                     const int64_t *__restrict__ gslice,
                                                     const int64_t *__restrict__ sptr, const int32_t *__restrict__ slot_row,
                                                     const int32_t *__restrict__ slot_len, const int32_t *__restrict__ col,
                                                     const double *__restrict__ val, const double *__restrict__ sdinv,
                                                     const double *b, double *y) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    const int64_t g0 = goff[blockIdx.x], g1 = goff[blockIdx.x + 1];
    for (int64_t g = g0; g < g1; ++g) {
        const int64_t s1 = gslice[g + 1];
        for (int64_t sl = gslice[g] + wave; sl < s1; sl += nw)
            tri_slice<4>(sl, lane, sptr, slot_row, slot_len, col, val, sdinv, b, y);
        __syncthreads();
    }
}

// one launch per group (global levels): slices [s0, s1)
__global__ __launch_bounds__(TPB) void k_tri_group(int64_t s0, int64_t s1, const int64_t *__restrict__ sptr,
                                                   const int32_t *__restrict__ slot_row,
                                                   const int32_t *__restrict__ slot_len, const int32_t *__restrict__ col,
                                                   const double *__restrict__ val, const double *__restrict__ sdinv,
                                                   const double *b, double *y) {
    const int lane = threadIdx.x & 63;
    const int64_t sl = s0 + (((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6);
    if (sl >= s1) return;
    tri_slice<4>(sl, lane, sptr, slot_row, slot_len, col, val, sdinv, b, y);
}

void launch_tri_fill(int64_t nslices, const int32_t *slot_row, const int32_t *slot_len, const int64_t *rp,
                     const int32_t *ci, const double *lu, const int64_t *diag, const double *dinv, int upper,
                     const int64_t *sptr, int32_t *ocol, double *oval, double *odinv, hipStream_t st) {
    if (nslices > 0)
        k_tri_fill<<<grid_for(nslices * 64, TPB), TPB, 0, st>>>(nslices, slot_row, slot_len, rp, ci, lu, diag, dinv,
                                                                upper, sptr, ocol, oval, odinv);
}
void launch_tri_blocks(int64_t nblocks, const int64_t *goff, const int64_t *gslice, const int64_t *sptr,
                       const int32_t *slot_row, const int32_t *slot_len, const int32_t *col, const double *val,
                       const double *sdinv, const double *b, double *y, hipStream_t st) {
    if (nblocks > 0)
        k_tri_blocks<<<(unsigned)nblocks, 1024, 0, st>>>(goff, gslice, sptr, slot_row, slot_len, col, val, sdinv, b, y);
}
// One level of a triangular sweep straight from the factored CSR: TRI_G lanes
// per row (entries dealt round robin, partial sums combined by lane shuffles),
// so a long row costs one or two dependent gather rounds instead of one per
// entry as with a lane per row.  upper = 0: y_i = b_i - sum_{k < diag} l_ik y_k;
// 1: y_i = dinv_i (b_i - sum_{k > diag} u_ik y_k) (b may alias y).
static constexpr int TRI_G = 16;
__global__ __launch_bounds__(TPB) void k_tri_csr_level(int64_t m, const int32_t *__restrict__ rows,
                                                       const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                       const double *__restrict__ val, const int64_t *__restrict__ diag,
                                                       const double *__restrict__ dinv, int upper, const double *b,
                                                       double *y) {
    const int64_t gid = (int64_t)blockIdx.x * TPB + threadIdx.x;
    const int64_t r = gid / TRI_G;
    const int j = (int)(gid % TRI_G);
    if (r >= m) return;  // whole groups of TRI_G lanes (m rows x TRI_G lanes, TRI_G divides 64)
    const int64_t i = rows[r], d = diag[i];
    const int64_t lo = upper ? d + 1 : rp[i], hi = upper ? rp[i + 1] : d;
    double s = 0.0;
    for (int64_t k = lo + j; k < hi; k += TRI_G) s += val[k] * y[ci[k]];
#pragma unroll
    for (int off = TRI_G / 2; off >= 1; off >>= 1) s += __shfl_xor(s, off, TRI_G);
    if (j == 0) {
        const double v = b[i] - s;
        y[i] = upper ? v * dinv[i] : v;
    }
}
void launch_tri_csr_level(int64_t m, const int32_t *rows, const int64_t *rp, const int32_t *ci, const double *val,
                          const int64_t *diag, const double *dinv, int upper, const double *b, double *y,
                          hipStream_t st) {
    if (m > 0)
        k_tri_csr_level<<<grid_for(m * TRI_G, TPB), TPB, 0, st>>>(m, rows, rp, ci, val, diag, dinv, upper, b, y);
}
void launch_tri_group(int64_t s0, int64_t s1, const int64_t *sptr, const int32_t *slot_row, const int32_t *slot_len,
                      const int32_t *col, const double *val, const double *sdinv, const double *b, double *y,
                      hipStream_t st) {
    if (s1 > s0)
        k_tri_group<<<grid_for((s1 - s0) * 64, TPB), TPB, 0, st>>>(s0, s1, sptr, slot_row, slot_len, col, val, sdinv,
                                                                   b, y);
}

// Block-Jacobi ILU(0) apply with the block's solution resident in LDS: the
// truncated factors only reference rows of their own block, so one workgroup
// loads x[b0, b0+len) into LDS, runs every forward level then every backward
// level against LDS (gathers and updates never leave the CU), and writes the
// block of y once.  Blocks are launched heaviest-last-index first (the
// pressure blocks at the end of the fp ordering carry the most levels).
// ------------------------------------------------ LDS sweep stream layout --
// The block-Jacobi LDS kernel reads each level's slices as streams.  A block
// whose rows are long gives each row LPR = 2 or 4 lanes (8 or 16 in the
// y-resident variant; entries dealt round robin, partial sums combined with
// lane shuffles), so every lane's share fits the P entries the pipeline keeps
// in registers; short-row blocks keep LPR = 1.  Slice = 64 / LPR rows of one
// level.  Entry 0 of every lane is a header -- col = (row - b0) | (entries of
// this lane << SW_ROW_BITS) (row SW_ROW_PAD: padding; 14 bits hold the
// longest row, ilu0_max_row()), val = 1/U_ii (upper factor) -- entries 1..L the lane's factor
// entries with block-local columns.  The only metadata a level needs is where
// its slice starts, known 64 levels ahead (see sweep2), so loads are issued D
// levels before use without a dependent metadata hop.
static constexpr int SW_ROW_BITS = 18;
static constexpr int32_t SW_ROW_PAD = (1 << SW_ROW_BITS) - 1;  // local rows 0..262,142

__global__ __launch_bounds__(TPB) void k_lds_fill(int64_t nslices, const int32_t *s_start, const int32_t *s_n,
                                                  const int32_t *s_lpr, const int32_t *order, const int64_t *rp,
                                                  const int32_t *ci, const double *lu, const int64_t *diag,
                                                  const double *dinv, int upper, int64_t n, int64_t nb,
                                                  const int64_t *sptr2, int32_t *ocol, double *oval, int wide,
                                                  const int32_t *posof, const int32_t *row_lo, const int64_t *bstart) {
    const int64_t sl = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (sl >= nslices) return;
    const int lpr = s_lpr[sl];
    const int r = lane / lpr, sub = lane % lpr;
    const int64_t i = r < s_n[sl] ? order[s_start[sl] + r] : -1;
    const int64_t base = sptr2[sl], L = (sptr2[sl + 1] - base) >> 6;
    int64_t b0 = 0, src = 0, len = 0;
    if (i >= 0) {
        int64_t blen;
        block_of(i, n, nb, bstart, b0, blen);
        src = upper ? diag[i] + 1 : rp[i];
        len = upper ? rp[i + 1] - diag[i] - 1 : diag[i] - rp[i];
    }
    const int64_t mine = len > sub ? (len - sub + lpr - 1) / lpr : 0;
    // posof (ring sweep): rows and columns become block-local positions in the
    // triangle's level order
    const int32_t me = i >= 0 ? (posof ? posof[i] : (int32_t)(i - b0)) : -1;
    // a padding lane's entries (value 0) read the slice's first row: in the
    // ring sweep that position is in the LDS ring, never a global fallback
    const int32_t pad = posof ? posof[order[s_start[sl]]] : 0;
    if (row_lo) {
        // ring sweep: only the row's near entries (position >= row_lo[i], in the
        // LDS ring when the row runs), dealt round robin over its lanes; the far
        // ones are applied to the row's input when its chunk is loaded.  Lane-
        // major layout: entry k of this lane at base + lane * L + k.
        const int32_t lo = i >= 0 ? row_lo[i] : 0;
        const int64_t lb = base + (int64_t)lane * L;
        ocol[lb] = me;
        oval[lb] = (upper && i >= 0) ? dinv[i] : 0.0;
        int64_t k = 1, m = 0;
        for (int64_t j = 0; j < len; ++j) {
            const int32_t pc = posof[ci[src + j]];
            if (pc < lo) continue;
            if (m++ % lpr != sub) continue;
            ocol[lb + k] = pc;
            oval[lb + k] = lu[src + j];
            ++k;
        }
        for (; k < L; ++k) {
            ocol[lb + k] = i >= 0 ? me : pad;
            oval[lb + k] = 0.0;
        }
        return;
    }
    ocol[base + lane] = wide ? me : (i >= 0 ? me : SW_ROW_PAD) | (int32_t)(mine << SW_ROW_BITS);
    oval[base + lane] = (upper && i >= 0) ? dinv[i] : 0.0;
    for (int64_t k = 1; k < L; ++k) {
        const int64_t j = (k - 1) * lpr + sub, pos = base + k * 64 + lane;
        ocol[pos] = j < len ? (posof ? posof[ci[src + j]] : (int32_t)(ci[src + j] - b0)) : (wide && i >= 0 ? me : pad);
        oval[pos] = j < len ? lu[src + j] : 0.0;
    }
}
void launch_lds_fill(int64_t nslices, const int32_t *s_start, const int32_t *s_n, const int32_t *s_lpr,
                     const int32_t *order, const int64_t *rp, const int32_t *ci, const double *lu, const int64_t *diag,
                     const double *dinv, int upper, int64_t n, int64_t nb, const int64_t *sptr2, int32_t *ocol,
                     double *oval, hipStream_t st, bool wide, const int32_t *posof, const int32_t *row_lo,
                     const int64_t *bstart) {
    if (nslices > 0)
        k_lds_fill<<<grid_for(nslices * 64, TPB), TPB, 0, st>>>(nslices, s_start, s_n, s_lpr, order, rp, ci, lu, diag,
                                                                dinv, upper, n, nb, sptr2, ocol, oval, wide ? 1 : 0,
                                                                posof, row_lo, bstart);
}

// One sweep over a block's levels.  Pipeline: the loads of level g+2 are
// issued while level g computes; slots live in a ring of 3 register sets
// indexed by compile-time constants (a register copy with a load in flight
// would make the compiler drain vmcnt to 0 every level).  Slice starts for 64
// levels come from vector registers (lane l: level gbase + l) filled by one
// gather per 62 levels and read with v_readlane -- no scalar loads in the
// loop, whose lgkmcnt waits would be paid at every LDS access.
template <int P>
struct Sw2Slot {
    int32_t c[P + 1];
    double v[P + 1];
    int64_t base, L;  // L: entries incl. header; base < 0: this wave has no slice
    int l2;           // ring sweep: log2 of the slice's lanes per row (slice starts carry it in bits 0-2)
};

__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
    const int32_t lo = __builtin_amdgcn_readlane((int32_t)(uint32_t)(uint64_t)v, l);
    const int32_t hi = __builtin_amdgcn_readlane((int32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// Ring sweep (R): the block solution lives in level-order position space; the
// last RING_SLOTS positions sit in an LDS ring (slot p % RING_SLOTS), older
// ones (far dependencies) were subtracted from the row's input when its chunk
// loaded (from the position-ordered global copy ypos).  Positions are
// processed in chunks of at most RING_CHUNK (level-aligned): at a chunk's first
// level its inputs are loaded into their ring slots, after which every
// position >= lo_ok = chunk end - RING_SLOTS is still in the ring.
// diagnostics (pls.ring_probe; timing only, wrong results): bit 0 -- factor loads
// range-checked away, bit 1 -- no compute, bit 2 -- no prefetch instructions
__constant__ int ring_probe;
static constexpr int RING_SLOTS = 16384;
static constexpr int RING_CHUNK = 4096;
struct RingIn {
    const int64_t *cg, *cp;   // per chunk: first level (group) / [start, end) positions (cp[2k], cp[2k+1])
    const int32_t *src_idx;   // per position: index of its input value in src (block offset b0 included)
    const double *src;        // L: x; U: the L sweep's ypos
    const int64_t *frp;       // far dependencies per position (b0 + p): CSR row pointers
    const int32_t *fcol;      // ... their block-local positions
    const double *fval;       // ... factor values
};
struct Sw2Ctx {
    const int64_t *gslice, *sptr;
    const int32_t *col;
    const double *val;
    double *ys;
    int64_t g1, gbase;
    int64_t gv, sb, se;  // lane l: gslice[gbase+l], sptr[gslice+wave], sptr[gslice+wave+1] (-1: none)
    int lane, wave, nw;
    bool upper;
    // ring sweep only
    double *ring, *ypos;     // LDS ring; this sweep's position-ordered output (block offset applied)
    int64_t lo_ok, ck, cend, cnext, b0, ck0;
    RingIn rin;
    __device__ __forceinline__ void refill(int64_t g) {
        gbase = g;
        const int64_t k = g + lane;
        const int64_t kc = k < g1 ? k : g1;
        gv = gslice[kc];
        const int64_t gn = gslice[kc + 1 <= g1 ? kc + 1 : g1];
        const int64_t sl = gv + wave;
        const bool ok = k < g1 && sl < gn;
        sb = ok ? sptr[sl] : -1;
        se = ok ? sptr[sl + 1] : -1;
        // consume the loads here: otherwise every level's v_readlane of these
        // registers inherits the refill path's "load pending" state and the
        // compiler drains vmcnt to 0 at each level, exposing all prefetches
        asm volatile("" : "+v"(gv), "+v"(sb), "+v"(se));
    }
};

template <int P, bool R>
__device__ __forceinline__ void sw2_issue(Sw2Ctx &x, int64_t g, Sw2Slot<P> &s) {
    const int l = (int)(g - x.gbase);
    int64_t base = g < x.g1 ? readlane64(x.sb, l) : -1;
    int64_t next = base >= 0 ? readlane64(x.se, l) : 0;
    s.l2 = 0;
    if (R) {  // slice starts are multiples of 64 entries; bits 0-2: log2(lanes per row)
        s.l2 = base >= 0 ? (int)(base & 7) : 0;
        base = base >= 0 ? (base & ~(int64_t)63) : -1;
        next &= ~(int64_t)63;
    }
    const int64_t L = base >= 0 ? (next - base) >> 6 : 0;
    s.base = base;
    s.L = L;
    if (R && (ring_probe & 4)) {  // diagnostics: no prefetch at all
        s.base = base;
#pragma unroll
        for (int u = 0; u <= P; ++u) { s.c[u] = 0; s.v[u] = 0.0; }
        return;
    }
    if (R) {
        // ring sweep: buffer loads through per-slot descriptors bounded to the
        // slice (0 bytes for an idle wave): entries past the slice and idle
        // waves' loads are range-checked away (no traffic, reads return 0),
        // and every path issues the same loads, which keeps the compiler's
        // vmcnt bookkeeping exact -- using this slot two levels later waits for
        // its own loads only (a branch around them made it wait for everything
        // in flight, the prefetch issued this level included)
        static_assert((P + 1) % 8 == 0, "the ring sweep's slot is one lane's first P + 1 entries (a multiple of 8)");
        const int64_t b = base >= 0 ? base : 0;
        const int nc = (base >= 0 && !(ring_probe & 1)) ? (int)(L * 64 * 4) : 0;
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void *)(x.col + b), (short)0, nc, 0x00020000);
        const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void *)(x.val + b), (short)0, 2 * nc, 0x00020000);
        const int off = x.lane * (int)L;  // lane-major, L a multiple of P + 1
#pragma unroll
        for (int q = 0; q < (P + 1) / 4; ++q) {
            const auto c4 = __builtin_amdgcn_raw_buffer_load_b128(rc, (off + 4 * q) * 4, 0, 0);
            s.c[4 * q + 0] = (int32_t)c4[0];
            s.c[4 * q + 1] = (int32_t)c4[1];
            s.c[4 * q + 2] = (int32_t)c4[2];
            s.c[4 * q + 3] = (int32_t)c4[3];
        }
#pragma unroll
        for (int q = 0; q < (P + 1) / 2; ++q) {
            const auto v4 = __builtin_amdgcn_raw_buffer_load_b128(rv, (off + 2 * q) * 8, 0, 0);
            s.v[2 * q + 0] = __builtin_bit_cast(double, ((uint64_t)v4[1] << 32) | v4[0]);
            s.v[2 * q + 1] = __builtin_bit_cast(double, ((uint64_t)v4[3] << 32) | v4[2]);
        }
        return;
    }
    if (base < 0) {  // wave idle at this level: no loads (they would only queue in the CU's memory pipe)
#pragma unroll
        for (int u = 0; u <= P; ++u) {
            s.c[u] = 0;
            s.v[u] = 0.0;
        }
        return;
    }
#pragma unroll
    for (int u = 0; u <= P; ++u) {
        const int64_t pos = base + (u < L ? u : 0) * 64 + x.lane;
        s.c[u] = __builtin_nontemporal_load(x.col + pos);
        s.v[u] = __builtin_nontemporal_load(x.val + pos);
    }
}

// W (wide, the y-resident sweep): header col = local row (-1: padding lane),
// a lane's padding entries point at its own row with value 0, so only the
// slice length masks entries and blocks may have up to 2^31 rows.
// the value of a dependency (block-local row, or position in the ring sweep)
template <bool R>
__device__ __forceinline__ double sw2_dep(const Sw2Ctx &x, int32_t c) {
    // ring sweep: every stream entry is a near dependency, in the LDS ring (no
    // global load in the level loop: vmcnt waits would drain the prefetches)
    if (R) return x.ring[c & (RING_SLOTS - 1)];
    return x.ys[c];
}

// a double through a DPP lane permutation (no LDS round trip, unlike a shuffle)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// index of entry k of a lane's stream: [k][lane] (LDS / y-resident sweeps) or,
// in the ring sweep, lane-major [lane][k] with L (a multiple of 8) entries per
// lane, so a slot's first 8 columns / values are 2 / 4 16-byte loads
template <bool R>
__device__ __forceinline__ int64_t sw2_at(int64_t base, int64_t L, int lane, int64_t k) {
    return R ? base + (int64_t)lane * L + k : base + k * 64 + lane;
}

// LPR = 0: lanes per row chosen per slice (ring sweep), 1 << l2
template <int LPR, bool W, bool R>
__device__ __forceinline__ void sw2_finish(const Sw2Ctx &x, int32_t h, double dv, double acc, int l2 = 0) {
    // the LPR partial sums of a row: quad_perm xor 1, xor 2, then row_half_mirror
    // and row_mirror -- after the quad steps every lane of a quad holds the same
    // value, so mirroring pairs exactly the sums xor 4 / xor 8 would (a + b =
    // b + a: bitwise the shuffle tree), without LDS round trips
    const int lg = LPR ? (LPR >= 32 ? 5 : LPR >= 16 ? 4 : LPR >= 8 ? 3 : LPR >= 4 ? 2 : LPR >= 2 ? 1 : 0) : l2;
    if (lg >= 1) acc += dpp_d<0xB1>(acc);
    if (lg >= 2) acc += dpp_d<0x4E>(acc);
    if (lg >= 3) acc += dpp_d<0x141>(acc);
    if (lg >= 4) acc += dpp_d<0x140>(acc);
    if (lg >= 5) acc += __shfl_xor(acc, 16);
    const int32_t li = W ? h : (h & SW_ROW_PAD);
    if ((x.lane & ((1 << lg) - 1)) == 0 && (W ? li >= 0 : li != SW_ROW_PAD)) {
        if (R) {  // li: the row's position; its input sits in its ring slot
            double *slot = x.ring + (li & (RING_SLOTS - 1));
            *slot = x.upper ? (*slot - acc) * dv : *slot - acc;  // to ypos in bulk at the next chunk
        } else {
            x.ys[li] = x.upper ? (x.ys[li] - acc) * dv : x.ys[li] - acc;
        }
    }
}

template <int LPR, bool W, bool R>
__device__ __forceinline__ void sw2_slice_inline(const Sw2Ctx &x, int64_t sl) {
    const int64_t enc = x.sptr[sl];
    const int64_t base = R ? (enc & ~(int64_t)63) : enc;
    const int64_t L = ((R ? (x.sptr[sl + 1] & ~(int64_t)63) : x.sptr[sl + 1]) - base) >> 6;
    const int32_t h = x.col[sw2_at<R>(base, L, x.lane, 0)];
    const double dv = x.val[sw2_at<R>(base, L, x.lane, 0)];
    const int32_t len = (int32_t)((uint32_t)h >> SW_ROW_BITS);
    double acc = 0.0;
    for (int64_t k = 1; k < L; ++k) {
        const int64_t pos = sw2_at<R>(base, L, x.lane, k);
        const int32_t cc = x.col[pos];
        const double vv = x.val[pos];
        if (W || k <= len) acc += __dmul_rn(vv, sw2_dep<R>(x, cc));
    }
    sw2_finish<LPR, W, R>(x, h, dv, acc, R ? (int)(enc & 7) : 0);
}

// ring sweep: results of positions [p0, p1) from the ring to ypos (they stay in
// the ring for RING_SLOTS - RING_CHUNK >= RING_CHUNK more positions)
__device__ __forceinline__ void ring_flush(Sw2Ctx &x, int64_t p0, int64_t p1) {
    for (int64_t t = p0 + threadIdx.x; t < p1; t += blockDim.x) x.ypos[t] = x.ring[t & (RING_SLOTS - 1)];
}

// ring sweep: at the first level of a chunk, the previous chunk's results to
// ypos, then this chunk's inputs into the ring
__device__ __forceinline__ void ring_chunk(Sw2Ctx &x, int64_t g) {
    if (g != x.cnext) return;
    if (x.ck > x.ck0) ring_flush(x, x.rin.cp[2 * x.ck - 2], x.rin.cp[2 * x.ck - 1]);
    const int64_t c0 = x.rin.cp[2 * x.ck], c1 = x.rin.cp[2 * x.ck + 1];
    for (int64_t t = c0 + threadIdx.x; t < c1; t += blockDim.x) {
        double v = x.rin.src[x.rin.src_idx[x.b0 + t]];
        // far dependencies (older than the ring keeps, final before this chunk),
        // eight at a time: their column / value loads, then their eight ypos
        // gathers, are all in flight before the subtractions, which run in the
        // stream's order (one entry at a time, every load waited for in turn,
        // was ~2 global latencies per far entry -- most of the N=24 sweep's
        // skeleton time)
        const int64_t e0 = x.rin.frp[x.b0 + t], e1 = x.rin.frp[x.b0 + t + 1];
        if (ring_probe & 64) {  // (diagnostics: the one-at-a-time loop, for A/B timing)
            for (int64_t e = e0; e < e1; ++e) v -= x.rin.fval[e] * x.ypos[x.rin.fcol[e]];
            x.ring[t & (RING_SLOTS - 1)] = v;
            continue;
        }
        for (int64_t e = e0; e < e1; e += 8) {
            int32_t fc[8];
            double fv[8], yv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t k = e + u < e1 ? e + u : e0;
                fc[u] = x.rin.fcol[k];
                fv[u] = x.rin.fval[k];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) yv[u] = x.ypos[fc[u]];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (e + u < e1) v -= fv[u] * yv[u];
        }
        x.ring[t & (RING_SLOTS - 1)] = v;
    }
    __syncthreads();
    x.lo_ok = c1 - RING_SLOTS;
    ++x.ck;
    x.cnext = x.ck < x.cend ? x.rin.cg[x.ck] : INT64_MAX;
}

template <int P, int LPR, bool W, bool R, int D = 2>
__device__ __forceinline__ void sw2_level(Sw2Ctx &x, int64_t g, const Sw2Slot<P> &cur, Sw2Slot<P> &ahead) {
    if (R) ring_chunk(x, g);
    if (g + D >= x.gbase + 64) x.refill(g);
    sw2_issue<P, R>(x, g + D, ahead);
    if (cur.base >= 0 && !(R && (ring_probe & 2))) {  // (probe bit 1: no compute, diagnostics)
        const int32_t h = cur.c[0];
        const int32_t len = W ? (int32_t)cur.L - 1 : (int32_t)((uint32_t)h >> SW_ROW_BITS);
        double acc = 0.0, d[P + 1];
        // every dependency read issued before the first is consumed (they are
        // independent; consuming in turn would serialise the LDS / L1 round trips)
        if (R) {
            // ring sweep: entries past the slice were range-checked to col 0 /
            // value 0 and padding entries carry value 0 on a written position,
            // so no masking: 0 * (a finite ring value) adds nothing
#pragma unroll
            for (int u = 1; u <= P; ++u) d[u] = sw2_dep<R>(x, cur.c[u]);
#pragma unroll
            for (int u = 1; u <= P; ++u) acc += __dmul_rn(cur.v[u], d[u]);  // no FMA: the other sweeps' rounding
        } else {
#pragma unroll
            for (int u = 1; u <= P; ++u) d[u] = sw2_dep<R>(x, u <= len ? cur.c[u] : 0);
#pragma unroll
            for (int u = 1; u <= P; ++u) {
                const double t = __dmul_rn(cur.v[u], d[u]);
                acc += (u <= len) ? t : 0.0;
            }
        }
        for (int64_t k0 = P + 1; k0 < cur.L; k0 += 8) {  // lanes with more than P entries: chunks of 8
            int32_t cc[8];
            double vv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t k = k0 + u < cur.L ? k0 + u : cur.L - 1;
                cc[u] = __builtin_nontemporal_load(x.col + sw2_at<R>(cur.base, cur.L, x.lane, k));
                vv[u] = __builtin_nontemporal_load(x.val + sw2_at<R>(cur.base, cur.L, x.lane, k));
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const double t = __dmul_rn(vv[u], sw2_dep<R>(x, k0 + u <= len ? cc[u] : 0));
                acc += (k0 + u <= len) ? t : 0.0;
            }
        }
        sw2_finish<LPR, W, R>(x, h, cur.v[0], acc, cur.l2);
        // levels with more slices than waves: the rest inline
        const int l = (int)(g - x.gbase);
        const int64_t s0 = readlane64(x.gv, l), s1 = readlane64(x.gv, l + 1);
        for (int64_t sl = s0 + x.wave + x.nw; sl < s1; sl += x.nw) sw2_slice_inline<LPR, W, R>(x, sl);
    }
    __syncthreads();
}

// D > 2: D levels of factor data in flight (D + 1 register slots, indexed by
// compile-time constants in the unrolled loop) -- for narrow levels under
// concurrent HBM traffic, where a load's latency exceeds two levels' time
template <int P, int LPR, bool W, int D>
__device__ __forceinline__ void sweep2_deep(Sw2Ctx &x, int64_t g0) {
    x.refill(g0);
    Sw2Slot<P> s[D + 1];
#pragma unroll
    for (int k = 0; k < D; ++k) sw2_issue<P, false>(x, g0 + k, s[k]);
    for (int64_t g = g0;;) {
#pragma unroll
        for (int k = 0; k <= D; ++k) {
            sw2_level<P, LPR, W, false, D>(x, g, s[k], s[(k + D) % (D + 1)]);
            if (++g >= x.g1) return;
        }
    }
}

template <int P, int LPR, bool W, bool R, int D = 2>
__device__ __forceinline__ void sweep2(Sw2Ctx &x, int64_t g0) {
    if (D != 2 && !R) {
        sweep2_deep<P, LPR, W, D>(x, g0);
        return;
    }
    x.refill(g0);
    Sw2Slot<P> s0, s1, s2;
    sw2_issue<P, R>(x, g0, s0);
    sw2_issue<P, R>(x, g0 + 1, s1);
    for (int64_t g = g0;;) {
        sw2_level<P, LPR, W, R>(x, g, s0, s2);
        if (++g >= x.g1) break;
        sw2_level<P, LPR, W, R>(x, g, s1, s0);
        if (++g >= x.g1) break;
        sw2_level<P, LPR, W, R>(x, g, s2, s1);
        if (++g >= x.g1) break;
    }
}

// Round-robin sweep for deep, narrow level DAGs (about one slice per level:
// FE rows in their natural order, e.g. the classical AMG's hybrid Gauss-Seidel
// chunks).  sweep2 gives every level to all waves and keeps two levels of
// factor data in flight, so with one slice per level one wave works, the rest
// idle at the barrier, and memory latency is exposed (footing N=128 smoother:
// ~0.77 us per level, 970 levels per 2,405-row chunk).  Here wave w owns the
// levels g0 + w, g0 + w + nw, ... and loads its next level's slice before
// computing the current one, so its data has nw levels' time to arrive.  A
// level's extra slices (rare) run inline.  Per-row sums are sweep2's (same
// entries, same order): results are bitwise those of sweep2.
// S > 1 (levels of a few slices: the pressure blocks of the headline's fp
// block, ~2 slices per level): groups of S waves own the levels round robin,
// wave k of a group the level's slice k, so data has nw / S levels to arrive.
template <int P, int LPR, bool W>
__device__ __forceinline__ void sweep_rr(Sw2Ctx &x, int64_t g0, int S = 1) {
    const int64_t g1 = x.g1;
    const int ng = x.nw / S, w = x.wave / S, ks = x.wave % S;  // level groups; this wave's group / slice
    const int nw = ng;
    const int64_t nown = g1 - g0 > w ? (g1 - g0 - w + nw - 1) / nw : 0;  // own levels of this wave
    int64_t jb = 0, ms0 = 0, ms1 = 0, mb = -1, me = -1;  // lane l: own level jb + l (first slice, end, entry range)
    auto refill = [&](int64_t j0) {
        jb = j0;
        const int64_t g = g0 + w + (j0 + x.lane) * nw;
        if (j0 + x.lane < nown) {
            ms0 = x.gslice[g];
            ms1 = x.gslice[g + 1];
            mb = ms1 > ms0 + ks ? x.sptr[ms0 + ks] : -1;
            me = ms1 > ms0 + ks ? x.sptr[ms0 + ks + 1] : -1;
        } else {
            ms0 = ms1 = 0;
            mb = me = -1;
        }
        asm volatile("" : "+v"(ms0), "+v"(ms1), "+v"(mb), "+v"(me));
    };
    auto issue = [&](int64_t j, Sw2Slot<P> &sl) {
        const int l = (int)(j - jb);
        const int64_t base = j < nown ? readlane64(mb, l) : -1;
        const int64_t next = base >= 0 ? readlane64(me, l) : 0;
        sl.base = base;
        sl.L = base >= 0 ? (next - base) >> 6 : 0;
        sl.l2 = 0;
#pragma unroll
        for (int u = 0; u <= P; ++u) {
            const int64_t pos = (base >= 0 ? base : 0) + (u < sl.L ? u : 0) * 64 + x.lane;
            sl.c[u] = base >= 0 ? __builtin_nontemporal_load(x.col + pos) : 0;
            sl.v[u] = base >= 0 ? __builtin_nontemporal_load(x.val + pos) : 0.0;
        }
    };
    auto compute = [&](int64_t j, const Sw2Slot<P> &cur) {
        if (cur.base < 0) return;
        const int32_t h = cur.c[0];
        const int32_t len = W ? (int32_t)cur.L - 1 : (int32_t)((uint32_t)h >> SW_ROW_BITS);
        double acc = 0.0, d[P + 1];
#pragma unroll
        for (int u = 1; u <= P; ++u) d[u] = sw2_dep<false>(x, u <= len ? cur.c[u] : 0);
#pragma unroll
        for (int u = 1; u <= P; ++u) {
            const double t = __dmul_rn(cur.v[u], d[u]);  // sweep2's rounding (no contraction)
            acc += (u <= len) ? t : 0.0;
        }
        for (int64_t k0 = P + 1; k0 < cur.L; k0 += 8) {
            int32_t cc[8];
            double vv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t k = k0 + u < cur.L ? k0 + u : cur.L - 1;
                cc[u] = __builtin_nontemporal_load(x.col + cur.base + k * 64 + x.lane);
                vv[u] = __builtin_nontemporal_load(x.val + cur.base + k * 64 + x.lane);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const double t = __dmul_rn(vv[u], sw2_dep<false>(x, k0 + u <= len ? cc[u] : 0));
                acc += (k0 + u <= len) ? t : 0.0;
            }
        }
        sw2_finish<LPR, W, false>(x, h, cur.v[0], acc);
        const int l = (int)(j - jb);
        const int64_t s0 = readlane64(ms0, l), s1 = readlane64(ms1, l);
        for (int64_t sl = s0 + ks + S; sl < s1; sl += S) sw2_slice_inline<LPR, W, false>(x, sl);
    };
    Sw2Slot<P> A, B;
    refill(0);
    issue(0, A);
    int64_t j = 0;
    for (int64_t g = g0; g < g1; ++g) {
        if ((g - g0) % nw == w) {
            if (j + 1 - jb >= 64) {  // keep the current level's metadata: refill from j
                refill(j);
            }
            // compute first: its wait covers only the slot loaded nw levels ago, not
            // the loads issued now for the next own level
            if ((j & 1) == 0) {
                compute(j, A);
                issue(j + 1, B);
            } else {
                compute(j, B);
                issue(j + 1, A);
            }
            ++j;
        }
        __syncthreads();
    }
}

template <int P, bool W, bool R = false, int D = 2>
__device__ __forceinline__ void sweep_block(int64_t g0, int64_t g1, int lpr, int lane, int wave, int nw, bool upper,
                                            const int64_t *__restrict__ gslice, const int64_t *__restrict__ sptr,
                                            const int32_t *__restrict__ col, const double *__restrict__ val,
                                            double *ys, double *ring = nullptr, double *ypos = nullptr,
                                            int64_t b0 = 0, int64_t ck0 = 0, int64_t ck1 = 0, RingIn rin = {},
                                            int rr = 0) {
    if (g0 >= g1) return;
    Sw2Ctx x{gslice, sptr, col, val, ys, g1, 0, 0, 0, 0, lane, wave, nw, upper,
             ring, ypos, 0, ck0, ck1, ck0 < ck1 ? rin.cg[ck0] : INT64_MAX, b0, ck0, rin};
    if (!R && rr) {  // deep, narrow levels: round-robin over groups of rr waves (a power of two <= nw)
        const int S = rr <= nw ? rr : nw;
        if (W) {
            if (lpr == 16) sweep_rr<P, 16, W>(x, g0, S);
            else if (lpr == 8) sweep_rr<P, 8, W>(x, g0, S);
            else if (lpr == 4) sweep_rr<P, 4, W>(x, g0, S);
            else if (lpr == 2) sweep_rr<P, 2, W>(x, g0, S);
            else sweep_rr<P, 1, W>(x, g0, S);
        } else {
            if (lpr == 4) sweep_rr<P, 4, W>(x, g0, S);
            else if (lpr == 2) sweep_rr<P, 2, W>(x, g0, S);
            else sweep_rr<P, 1, W>(x, g0, S);
        }
        return;
    }
    if (R) {  // ring sweep: lanes per row per slice
        sweep2<P, 0, true, true>(x, g0);
        if (ck1 > ck0) ring_flush(x, rin.cp[2 * ck1 - 2], rin.cp[2 * ck1 - 1]);  // the last chunk
        return;
    }
    if (W) {  // the y-resident sweep: 8 / 16 lanes for long rows
        if (lpr == 16) sweep2<P, 16, W, R, D>(x, g0);
        else if (lpr == 8) sweep2<P, 8, W, R, D>(x, g0);
        else if (lpr == 4) sweep2<P, 4, W, R, D>(x, g0);
        else if (lpr == 2) sweep2<P, 2, W, R, D>(x, g0);
        else sweep2<P, 1, W, R, D>(x, g0);
        return;
    }
    if (lpr == 4) sweep2<P, 4, W, R, D>(x, g0);
    else if (lpr == 2) sweep2<P, 2, W, R, D>(x, g0);
    else sweep2<P, 1, W, R, D>(x, g0);
}

static constexpr int SW_P = 7;  // factor entries per lane kept in registers per pipeline slot
// the ring sweep's slot and workgroup (measured: 512 threads with 15-entry
// slots, which hold the wider N=20 levels without in-level reloads, were
// slower at both N=12 (93 vs 138 it/s) and N=20 (16.6 vs 23.2))
static constexpr int RING_P = 7, RING_TPB = 1024;

// GMEM: the block solution lives in y itself (global memory) instead of LDS --
// blocks longer than the LDS holds, with the wide slice headers (W).  All waves of the workgroup share the CU's
// vector L1, so y written by one wave before __syncthreads() is seen by the
// others after it (workgroup-scope coherence, no cache maintenance needed).
// D: levels of factor data in flight (2; deeper with fewer threads: TPBMAX)
template <bool GMEM, int D = 2, int TPBMAX = 1024>
__global__ __launch_bounds__(TPBMAX) void k_ilu_blocks_lds(int64_t n, int64_t nblocks, const int64_t *__restrict__ Lgoff,
                                                         const int64_t *__restrict__ Lgslice,
                                                         const int64_t *__restrict__ Lsptr,
                                                         const int32_t *__restrict__ Lcol,
                                                         const double *__restrict__ Lval,
                                                         const int32_t *__restrict__ Llpr,
                                                         const int64_t *__restrict__ Ugoff,
                                                         const int64_t *__restrict__ Ugslice,
                                                         const int64_t *__restrict__ Usptr,
                                                         const int32_t *__restrict__ Ucol,
                                                         const double *__restrict__ Uval,
                                                         const int32_t *__restrict__ Ulpr, const double *x,
                                                         double *y, int64_t *__restrict__ prof, int rr,
                                                         const int64_t *__restrict__ bstart, int64_t blk_hi) {
    extern __shared__ __attribute__((aligned(16))) double lds_y[];
    // blocks [blk_hi - gridDim.x, blk_hi), the last (heaviest) first
    const int64_t blk = blk_hi - 1 - (int64_t)blockIdx.x;
    int64_t b0, len;
    block_range(blk, n, nblocks, bstart, b0, len);
    double *ys = GMEM ? y + b0 : lds_y;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    int64_t t0 = 0, t1 = 0;
    if (prof) t0 = wall_clock64();
    if (!GMEM || x != y)
        for (int64_t t = threadIdx.x; t < len; t += blockDim.x) ys[t] = x[b0 + t];
    __syncthreads();
    sweep_block<SW_P, GMEM, false, D>(Lgoff[blk], Lgoff[blk + 1], Llpr[blk], lane, wave, nw, false, Lgslice, Lsptr, Lcol,
                                      Lval, ys, nullptr, nullptr, 0, 0, 0, {}, rr);
    if (prof) t1 = wall_clock64();
    sweep_block<SW_P, GMEM, false, D>(Ugoff[blk], Ugoff[blk + 1], Ulpr[blk], lane, wave, nw, true, Ugslice, Usptr, Ucol,
                                      Uval, ys, nullptr, nullptr, 0, 0, 0, {}, rr);
    if (!GMEM)
        for (int64_t t = threadIdx.x; t < len; t += blockDim.x) y[b0 + t] = ys[t];
    if (prof && threadIdx.x == 0) {  // diagnostics (option pls.sweep_profile): 100 MHz wall clock
        int64_t *p = prof + blk * 8;
        p[0] = t0;
        p[1] = t1;
        p[2] = wall_clock64();
        p[3] = Lgoff[blk + 1] - Lgoff[blk];
        p[4] = Ugoff[blk + 1] - Ugoff[blk];
        p[5] = len;
        p[6] = Lgslice[Lgoff[blk + 1]] - Lgslice[Lgoff[blk]];
        p[7] = Llpr[blk] * 10 + Ulpr[blk];
    }
}

// The ring sweep (whole FE blocks in a bandwidth-reducing order: deep, narrow
// level DAGs whose dependencies are recent in level order): per block, the L
// sweep in L's level-order positions (inputs x[ordL]), outputs to yL (position
// order); the U sweep in U's positions (inputs yL[mapUL]), outputs to yU; then
// y[ordU[p]] = yU[p].  Dependency reads hit the LDS ring unless older than
// RING_SLOTS - RING_CHUNK positions (then yL / yU in global memory, written by
// this workgroup: workgroup-scope coherence as in the y-resident sweep), and
// those "far" dependencies are known at setup: they are taken out of the
// factor streams and subtracted from the row's input when its chunk loads.
__global__ __launch_bounds__(RING_TPB) void k_ilu_blocks_ring(
    int64_t n, int64_t nblocks, const int64_t *__restrict__ Lgoff, const int64_t *__restrict__ Lgslice,
    const int64_t *__restrict__ Lsptr, const int32_t *__restrict__ Lcol, const double *__restrict__ Lval,
    const int32_t *__restrict__ Llpr, const int64_t *__restrict__ Ugoff, const int64_t *__restrict__ Ugslice,
    const int64_t *__restrict__ Usptr, const int32_t *__restrict__ Ucol, const double *__restrict__ Uval,
    const int32_t *__restrict__ Ulpr, const int64_t *__restrict__ Lcoff, const int64_t *__restrict__ Lcg,
    const int64_t *__restrict__ Lcp, const int64_t *__restrict__ Ucoff, const int64_t *__restrict__ Ucg,
    const int64_t *__restrict__ Ucp, const int32_t *__restrict__ ordL, const int32_t *__restrict__ mapUL,
    const int32_t *__restrict__ ordU, const int64_t *__restrict__ Lfrp, const int32_t *__restrict__ Lfcol,
    const double *__restrict__ Lfval, const int64_t *__restrict__ Ufrp, const int32_t *__restrict__ Ufcol,
    const double *__restrict__ Ufval, const double *x, double *y, double *yL, double *yU,
    const int64_t *__restrict__ bstart) {
    extern __shared__ __attribute__((aligned(16))) double ring[];
    const int64_t blk = nblocks - 1 - (int64_t)blockIdx.x;
    int64_t b0, len;
    block_range(blk, n, nblocks, bstart, b0, len);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    sweep_block<RING_P, true, true>(Lgoff[blk], Lgoff[blk + 1], Llpr[blk], lane, wave, nw, false, Lgslice, Lsptr, Lcol,
                                  Lval, nullptr, ring, yL + b0, b0, Lcoff[blk], Lcoff[blk + 1],
                                  RingIn{Lcg, Lcp, ordL, x, Lfrp, Lfcol, Lfval});
    __syncthreads();
    sweep_block<RING_P, true, true>(Ugoff[blk], Ugoff[blk + 1], Ulpr[blk], lane, wave, nw, true, Ugslice, Usptr, Ucol,
                                  Uval, nullptr, ring, yU + b0, b0, Ucoff[blk], Ucoff[blk + 1],
                                  RingIn{Ucg, Ucp, mapUL, yL, Ufrp, Ufcol, Ufval});
    __syncthreads();
    for (int64_t t = threadIdx.x; t < len; t += blockDim.x) y[ordU[b0 + t]] = yU[b0 + t];
}

void launch_ilu_blocks_ring(int64_t n, int64_t nblocks, const int64_t *Lgoff, const int64_t *Lgslice,
                            const int64_t *Lsptr, const int32_t *Lcol, const double *Lval, const int32_t *Llpr,
                            const int64_t *Ugoff, const int64_t *Ugslice, const int64_t *Usptr, const int32_t *Ucol,
                            const double *Uval, const int32_t *Ulpr, const int64_t *Lcoff, const int64_t *Lcg,
                            const int64_t *Lcp, const int64_t *Ucoff, const int64_t *Ucg, const int64_t *Ucp,
                            const int32_t *ordL, const int32_t *mapUL, const int32_t *ordU, const int64_t *Lfrp,
                            const int32_t *Lfcol, const double *Lfval, const int64_t *Ufrp, const int32_t *Ufcol,
                            const double *Ufval, const double *x, double *y, double *yL, double *yU, hipStream_t st,
                            int tpb, const int64_t *bstart) {
    if (tpb < 64 || tpb > RING_TPB || (tpb & 63)) tpb = RING_TPB;
    static bool configured = false;
    const int bytes = RING_SLOTS * 8;
    if (!configured) {
        (void)hipFuncSetAttribute((const void *)k_ilu_blocks_ring, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        configured = true;
    }
    k_ilu_blocks_ring<<<(unsigned)nblocks, tpb, bytes, st>>>(n, nblocks, Lgoff, Lgslice, Lsptr, Lcol, Lval, Llpr,
                                                               Ugoff, Ugslice, Usptr, Ucol, Uval, Ulpr, Lcoff, Lcg, Lcp,
                                                               Ucoff, Ucg, Ucp, ordL, mapUL, ordU, Lfrp, Lfcol, Lfval,
                                                               Ufrp, Ufcol, Ufval, x, y, yL, yU, bstart);
}
void set_ring_probe(int v) { (void)hipMemcpyToSymbol(HIP_SYMBOL(ring_probe), &v, sizeof(int)); }
int ilu_ring_slots() { return RING_SLOTS; }
int ilu_ring_lane_entries() { return RING_P; }
int ilu_ring_chunk() { return RING_CHUNK; }

int ilu_lds_max_rows() { return 163840 / 8; }
int ilu_gmem_max_rows() { return 0x7FFFFFFF; }
int ilu_lds_lane_entries() { return SW_P; }

void launch_ilu_blocks_lds(int64_t n, int64_t nblocks, const int64_t *Lgoff, const int64_t *Lgslice,
                           const int64_t *Lsptr, const int32_t *Lcol, const double *Lval, const int32_t *Llpr,
                           const int64_t *Ugoff, const int64_t *Ugslice, const int64_t *Usptr, const int32_t *Ucol,
                           const double *Uval, const int32_t *Ulpr, const double *x, double *y, hipStream_t st,
                           int64_t *prof, bool gmem, int tpb, int rr, const int64_t *bstart, int64_t max_len,
                           int64_t blk_lo, int64_t blk_hi, int depth) {
    // tpb: threads per workgroup, 64 .. 1024 (narrow levels: fewer waves, cheaper barriers)
    if (tpb < 64 || tpb > 1024 || (tpb & 63)) tpb = 1024;
    // block subset [blk_lo, blk_hi) (blk_hi < 0: every block)
    if (blk_hi < 0) {
        blk_lo = 0;
        blk_hi = nblocks;
    }
    if (blk_lo < 0 || blk_hi > nblocks || blk_lo >= blk_hi) return;
    const unsigned grid = (unsigned)(blk_hi - blk_lo);
    static bool configured = false;
    if (!configured) {
        (void)hipFuncSetAttribute((const void *)k_ilu_blocks_lds<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)163840);
        configured = true;
    }
    if (gmem) {
        k_ilu_blocks_lds<true><<<grid, tpb, 0, st>>>(n, nblocks, Lgoff, Lgslice, Lsptr, Lcol, Lval, Llpr, Ugoff, Ugslice,
                                                     Usptr, Ucol, Uval, Ulpr, x, y, prof, rr, bstart, blk_hi);
        return;
    }
    const size_t bytes = (size_t)(max_len > 0 ? max_len : n / nblocks + 1) * 8;
    if ((depth == 3 || depth == 4) && rr == 0) {  // 3 / 4 levels in flight on up to 16 waves (pls.sweep_depth)
        static bool conf34 = false;
        if (!conf34) {
            (void)hipFuncSetAttribute((const void *)k_ilu_blocks_lds<false, 3, 1024>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)163840);
            (void)hipFuncSetAttribute((const void *)k_ilu_blocks_lds<false, 4, 1024>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)163840);
            conf34 = true;
        }
        if (depth == 3)
            k_ilu_blocks_lds<false, 3, 1024><<<grid, tpb, bytes, st>>>(n, nblocks, Lgoff, Lgslice, Lsptr, Lcol, Lval,
                                                                       Llpr, Ugoff, Ugslice, Usptr, Ucol, Uval, Ulpr,
                                                                       x, y, prof, rr, bstart, blk_hi);
        else
            k_ilu_blocks_lds<false, 4, 1024><<<grid, tpb, bytes, st>>>(n, nblocks, Lgoff, Lgslice, Lsptr, Lcol, Lval,
                                                                       Llpr, Ugoff, Ugslice, Usptr, Ucol, Uval, Ulpr,
                                                                       x, y, prof, rr, bstart, blk_hi);
        return;
    }
    if (depth == 6 && tpb <= 512 && rr == 0) {  // 6 levels in flight, at most 8 waves (register room)
        static bool conf6 = false;
        if (!conf6) {
            (void)hipFuncSetAttribute((const void *)k_ilu_blocks_lds<false, 6, 512>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)163840);
            conf6 = true;
        }
        k_ilu_blocks_lds<false, 6, 512><<<grid, tpb, bytes, st>>>(n, nblocks, Lgoff, Lgslice, Lsptr, Lcol, Lval, Llpr,
                                                                 Ugoff, Ugslice, Usptr, Ucol, Uval, Ulpr, x, y, prof,
                                                                 rr, bstart, blk_hi);
        return;
    }
    k_ilu_blocks_lds<false><<<grid, tpb, bytes, st>>>(n, nblocks, Lgoff, Lgslice, Lsptr, Lcol, Lval, Llpr, Ugoff,
                                                        Ugslice, Usptr, Ucol, Uval, Ulpr, x, y, prof, rr, bstart, blk_hi);
}

// ======================================================= chain sweep ====
// Blocks whose level DAG is deep and narrow -- FE rows in their natural
// order, ~2-3 rows per level: the classical AMG's hybrid Gauss-Seidel chunks
// (footing's solid block, the synthetic N=59 s block) -- spend their time in
// the per-level hand-off, not in bytes: the workgroup sweep above pays a
// barrier and a two-level-deep prefetch per level (~0.77 us per level on the
// footing N=128 chunks).  Here ONE wave walks a block's rows in STEPS of one
// 16-lane DPP row each -- the rows of a step belong to one level, so they are
// independent; a level with more rows takes several steps, one after the
// other -- with no barrier (the LDS accesses of one wave complete in order).
// A slice packs up to 4 consecutive steps (lanes 16q .. 16q + 15: step q),
// and NW_D slices of factor data are in flight (6 loads each: the in-order
// vmcnt covers <= 63 outstanding), i.e. up to 32 steps of look-ahead.
//
// Stream layout (per triangle, runtime.cpp build_chain_tri): a slice is nl *
// L entries (nl = 16 x its steps, L = 8 entries per lane, lane-major), lane
// l's header (col = local row | count << SW_ROW_BITS, SW_ROW_PAD: no row; val
// = 1 / U_ii for the upper triangle) then its factor entries at l * L, unused
// ones (column 0, value 0: summed unmasked); slices follow one another, and a separate array holds every slice's size
// | (L == 8), read 64 slices at a time into a vector register (lane l: slice
// w0 + l) and picked with v_readlane.  A row's entries are dealt round robin
// over its LPR lanes and the partial sums combined by the DPP tree of
// sw2_finish, as in the LDS sweep: with the same lanes per row the results are
// bitwise those of k_ilu_blocks_lds.
static constexpr int NW_D = 8;  // slices in flight per wave
struct NwSlot {
    int32_t c[8];
    double v[8];
    int nl;  // active lanes of this slice (16 per step)
};

__device__ __forceinline__ void nw_issue(const int32_t *col, const double *val, int64_t base, int32_t szf, int lane,
                                         NwSlot &s, int probe) {
    const int L = (szf & 1) ? 8 : 4;
    s.nl = (szf & ~3) / L;
    const int sz = (probe & 16) ? 0 : (szf & ~3);  // (diagnostics: no factor traffic)
    // range-checked to the slice: lanes past nl and slices past the block's
    // end (size 0) read zeros without traffic; every path issues the same
    // 6 loads, so the compiler's vmcnt bookkeeping stays exact
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void *)(col + base), (short)0, sz * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void *)(val + base), (short)0, sz * 8, 0x00020000);
    const int off = lane * L;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const auto c4 = __builtin_amdgcn_raw_buffer_load_b128(rc, (off + 4 * q) * 4, 0, 0);
        s.c[4 * q + 0] = (int32_t)c4[0];
        s.c[4 * q + 1] = (int32_t)c4[1];
        s.c[4 * q + 2] = (int32_t)c4[2];
        s.c[4 * q + 3] = (int32_t)c4[3];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const auto v4 = __builtin_amdgcn_raw_buffer_load_b128(rv, (off + 2 * q) * 8, 0, 0);
        s.v[2 * q + 0] = __builtin_bit_cast(double, ((uint64_t)v4[1] << 32) | v4[0]);
        s.v[2 * q + 1] = __builtin_bit_cast(double, ((uint64_t)v4[3] << 32) | v4[2]);
    }
}

template <int LPR>
__device__ __forceinline__ void nw_compute(const NwSlot &s, double *ys, int lane, bool upper, int probe) {
    const int nsteps = s.nl >> 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // the slice's steps in order: step q is lanes 16q .. 16q + 15
        if (q < nsteps && (lane >> 4) == q) {
            const int32_t h = s.c[0];
            const int32_t li = h & SW_ROW_PAD;
            // the row's own input first, then every dependency read before the first is consumed
            const double yi = ys[li != SW_ROW_PAD ? li : 0];
            double acc = 0.0, d[8];
            // entries past a lane's count are stored as (column 0, value 0): no
            // per-entry masking, and 0 * y adds nothing (the LDS sweep's sums bitwise)
#pragma unroll
            for (int u = 1; u < 8; ++u) d[u] = ys[s.c[u]];
#pragma unroll
            for (int u = 1; u < 8; ++u) acc += __dmul_rn(s.v[u], d[u]);  // no contraction: the LDS sweep's rounding
            constexpr int lg = LPR >= 16 ? 4 : LPR >= 8 ? 3 : LPR >= 4 ? 2 : LPR >= 2 ? 1 : 0;
            if (lg >= 1) acc += dpp_d<0xB1>(acc);
            if (lg >= 2) acc += dpp_d<0x4E>(acc);
            if (lg >= 3) acc += dpp_d<0x141>(acc);
            if (lg >= 4) acc += dpp_d<0x140>(acc);
            if (!(probe & 32) && (lane & (LPR - 1)) == 0 && li != SW_ROW_PAD)
                ys[li] = upper ? (yi - acc) * s.v[0] : yi - acc;
        }
    }
}

// probe (pls.ring_probe bits 3 / 4 / 5; diagnostics, results wrong): no compute / no factor
// traffic / no LDS update of the row (no step waits on the previous one)
template <int LPR>
__device__ __forceinline__ void nw_sweep(int64_t base, const int32_t *sz, int64_t nsl, const int32_t *col,
                                         const double *val, double *ys, int lane, bool upper, int probe) {
    if (nsl <= 0) return;
    // slice sizes: lane l of `win` holds slice w0 + l, of `nxt` slice w0 + 64 + l
    // (loaded a window ahead, so picking from it never waits on a fresh load)
    int64_t w0 = 0;
    int32_t win = lane < nsl ? sz[lane] : 0;
    int32_t nxt = 64 + lane < nsl ? sz[64 + lane] : 0;
    auto size_of = [&](int64_t t) -> int32_t {
        if (t >= nsl) return 0;
        const int d = (int)(t - w0);
        return d < 64 ? __builtin_amdgcn_readlane(win, d) : __builtin_amdgcn_readlane(nxt, d - 64);
    };
    NwSlot s[NW_D];
    int64_t ib = base;  // where the next issued slice starts
#pragma unroll
    for (int k = 0; k < NW_D; ++k) {
        const int32_t f = size_of(k);
        nw_issue(col, val, ib, f, lane, s[k], probe);
        ib += f & ~3;
    }
    // whole rounds of NW_D slices without an exit inside (a loop exit between the
    // slots makes the compiler's vmcnt bookkeeping give up at the loop header and
    // drain every load in flight), then the last nsl % NW_D slices
    const int64_t rounds = nsl / NW_D;
    for (int64_t j = 0; j < rounds; ++j) {
        const int64_t t0 = (j + 1) * NW_D;  // first slice issued this round
        if (t0 >= w0 + 64) {  // move the window (the next one is loaded now, needed >= 7 rounds later)
            w0 += 64;
            win = nxt;
            nxt = w0 + 64 + lane < nsl ? sz[w0 + 64 + lane] : 0;
        }
#pragma unroll
        for (int k = 0; k < NW_D; ++k) {
            if (!(probe & 8)) nw_compute<LPR>(s[k], ys, lane, upper, probe);
            const int32_t f = size_of(t0 + k);
            nw_issue(col, val, ib, f, lane, s[k], probe);
            ib += f & ~3;
        }
    }
    const int rem = (int)(nsl - rounds * NW_D);
#pragma unroll
    for (int k = 0; k < NW_D; ++k)
        if (k < rem && !(probe & 8)) nw_compute<LPR>(s[k], ys, lane, upper, probe);
}

__device__ __forceinline__ void nw_dispatch(int lpr, int64_t base, const int32_t *sz, int64_t nsl,
                                            const int32_t *col, const double *val, double *ys, int lane, bool upper,
                                            int probe) {
    switch (lpr) {
        case 16: nw_sweep<16>(base, sz, nsl, col, val, ys, lane, upper, probe); break;
        case 8: nw_sweep<8>(base, sz, nsl, col, val, ys, lane, upper, probe); break;
        case 4: nw_sweep<4>(base, sz, nsl, col, val, ys, lane, upper, probe); break;
        case 2: nw_sweep<2>(base, sz, nsl, col, val, ys, lane, upper, probe); break;
        default: nw_sweep<1>(base, sz, nsl, col, val, ys, lane, upper, probe); break;
    }
}

__global__ __launch_bounds__(64) void k_ilu_blocks_chain(
    int64_t n, int64_t nblocks, const int64_t *__restrict__ bstart, const int64_t *__restrict__ Lbase,
    const int64_t *__restrict__ Lsoff, const int32_t *__restrict__ Lsz, const int64_t *__restrict__ Lnsl,
    const int32_t *__restrict__ Llpr,
    const int32_t *__restrict__ Lcol, const double *__restrict__ Lval, const int64_t *__restrict__ Ubase,
    const int64_t *__restrict__ Usoff, const int32_t *__restrict__ Usz, const int64_t *__restrict__ Unsl,
    const int32_t *__restrict__ Ulpr,
    const int32_t *__restrict__ Ucol, const double *__restrict__ Uval, const double *x, double *y) {
    extern __shared__ __attribute__((aligned(16))) double ys[];
    const int64_t blk = nblocks - 1 - (int64_t)blockIdx.x;  // heaviest (last) blocks first
    int64_t b0, len;
    block_range(blk, n, nblocks, bstart, b0, len);
    const int lane = threadIdx.x;
    for (int64_t t = lane; t < len; t += 64) ys[t] = x[b0 + t];
    __syncthreads();
    const int probe = __builtin_amdgcn_readfirstlane(ring_probe);
    nw_dispatch(Llpr[blk], Lbase[blk], Lsz + Lsoff[blk], Lnsl[blk], Lcol, Lval, ys, lane, false, probe);
    nw_dispatch(Ulpr[blk], Ubase[blk], Usz + Usoff[blk], Unsl[blk], Ucol, Uval, ys, lane, true, probe);
    __syncthreads();
    for (int64_t t = lane; t < len; t += 64) y[b0 + t] = ys[t];
}

int ilu_chain_depth() { return NW_D; }
int ilu_chain_max_lpr() { return 16; }

void launch_ilu_blocks_chain(int64_t n, int64_t nblocks, const int64_t *bstart, const int64_t *Lbase,
                             const int64_t *Lsoff, const int32_t *Lsz, const int64_t *Lnsl, const int32_t *Llpr,
                             const int32_t *Lcol, const double *Lval, const int64_t *Ubase, const int64_t *Usoff,
                             const int32_t *Usz, const int64_t *Unsl, const int32_t *Ulpr, const int32_t *Ucol,
                             const double *Uval, const double *x, double *y, int64_t max_len, hipStream_t st) {
    static bool configured = false;
    if (!configured) {
        (void)hipFuncSetAttribute((const void *)k_ilu_blocks_chain, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)163840);
        configured = true;
    }
    const size_t bytes = (size_t)std::max<int64_t>(max_len, 1) * 8;
    k_ilu_blocks_chain<<<(unsigned)nblocks, 64, bytes, st>>>(n, nblocks, bstart, Lbase, Lsoff, Lsz, Lnsl, Llpr, Lcol,
                                                             Lval, Ubase, Usoff, Usz, Unsl, Ulpr, Ucol, Uval, x, y);
}

// ============================================================ window sweep ====
// Triangular sweeps of LDS-resident blocks in windows of 64 consecutive rows
// (lane = row): y_w = T_w^-1 (b_w - A_{w,off} y_off) with T_w the window's
// diagonal block of the triangle (unit lower for L, with the diagonal for U)
// inverted once at setup and stored column-major ([k][lane]), and A_{w,off}
// the rows' entries outside the window on the solved side (SELL: [k][lane],
// block-local columns, padding = column 0 with value 0).  The dependent chain
// of a block is its windows (len / 64 steps of a 64 x 64 GEMV) instead of its
// levels: FE rows in natural order have ~1 row per level (the AMG smoother's
// chunks: ~970 levels per 2,405-row chunk, 38 windows).
// Four waves per block: wave q takes the stream entries k = q, q + 4, ... and
// the inverse's columns [16 q, 16 q + 16); the partial sums meet in LDS in a
// fixed order (two barriers per window).  Each wave prefetches its share of
// the next window (16 columns of T^-1, WIN_KPW stream entries per lane) into
// registers, reloading each right after its use with range-checked buffer
// loads (the zero triangle of T^-1 and entries past the window's stream read
// 0 without traffic), so a window's data was requested a window earlier and
// the register set stays small enough for the compiler to count the loads in
// flight.  (One wave with all 64 columns spilled to AGPRs and drained vmcnt at
// every window; staging through LDS by LDS-DMA cost ~4.4 us per window in
// 1-KiB copies.)  Rows have at most WIN_KP off-window entries (the setup
// keeps other blocks on the other sweeps), so every load is of fixed count.
static constexpr int WIN_NW = 4, WIN_KPW = 8;
static constexpr int WIN_KP = WIN_NW * WIN_KPW;  // stream entries per row (every one prefetched); blocks with more use other sweeps

// a block's window stream offsets, 64 per vector register (lane l: window j * 64 + l),
// picked with v_readlane: no scalar load (and its latency) per window
// (WIN_OFFR registers hold 64 * WIN_OFFR offsets: every window of a block up to
// ilu_window_max_rows() rows plus the end offset -- 312 for 19,904 rows)
static constexpr int WIN_OFFR = 5;
// the ring variant (blocks longer than LDS): offsets in LDS, up to 1,023 windows
static constexpr int WIN_OFFR_RING = 16, WIN_RING = 16384;
template <int R>
struct WinOff {
    int64_t r[R];
    __device__ __forceinline__ int64_t at(int64_t w) const {  // branch-free: R readlanes, scalar selects
        // (vector selects of the window's register and one readlane: the compiler
        // turned r[] into a scratch array indexed per window, whose loads drain
        // vmcnt -- the ring variant keeps its offsets in LDS instead)
        const int j = (int)(w >> 6), l = (int)(w & 63);
        int64_t v = readlane64(r[0], l);
#pragma unroll
        for (int k = 1; k < R; ++k) {
            const int64_t t = readlane64(r[k], l);
            v = j == k ? t : v;
        }
        return v;
    }
};

// a wave-uniform value forced into scalar registers (buffer resources must be SGPRs;
// without this the compiler may build them in VGPRs and waterfall every load)
__device__ __forceinline__ int64_t sgpr64(int64_t v) {
    const int32_t lo = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)(uint64_t)v);
    const int32_t hi = __builtin_amdgcn_readfirstlane((int32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t win_rsrc(const void *base, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)(uintptr_t)sgpr64((int64_t)(uintptr_t)base), (short)0,
                                             __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
}

typedef double win_d2 __attribute__((ext_vector_type(2)));
typedef int win_i3 __attribute__((ext_vector_type(3)));  // a stream record: value (lo, hi), column
template <int KPW>
struct WinBuf {  // one wave's share of a window's data in registers
    win_d2 tv[8];     // T^-1 columns 16 q + 2 j, + 1 of the lane's row
    win_i3 sr[KPW];   // stream records: value (.x lo, .y hi), column (.z)
    double rx;            // (ring variant) the window's input rows, from global memory
};

// Range-checked buffer loads (the inverse's column pairs 16 bytes, stream
// records 12) issued through inline asm: the compiler does not track them, so
// it cannot drain them at the loop header (its waits for loop-carried loads
// were vmcnt(0)); the sweep counts them itself -- every window issues the same
// number -- and win_wait ties the registers to the wait (no use or copy can
// move above it).  (Round 6: 8-byte loads, two per stream entry, were 33
// instructions per wave and window, and the loads -- whole wave-wide
// transfers: out-of-range or exec-masked lanes cost the same -- took ~1.1 of
// the ~1.9 us per window on the swelling N = 160 chunks.)
// (KPW: stream records per wave and window -- 4 where no row has more than 16
// off-window entries, else WIN_KPW.  Loading only the records inside each
// window's stream -- a wave-uniform count, waited for through a switch of
// vmcnt immediates -- was measured slower: 274 against 239 us per swelling
// N = 80 level-0 sweep, 1,420 against 1,361 at N = 160)
template <bool RING, int KPW>
constexpr int win_loads() { return 8 + KPW + (RING ? 1 : 0); }
__device__ __forceinline__ double win_ld64(__amdgpu_buffer_rsrc_t r, int off) {
    double v;
    asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r) : "memory");
    return v;
}
__device__ __forceinline__ win_d2 win_ld128(__amdgpu_buffer_rsrc_t r, int off) {
    win_d2 v;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r) : "memory");
    return v;
}
__device__ __forceinline__ win_i3 win_ld96(__amdgpu_buffer_rsrc_t r, int off) {
    win_i3 v;
    asm volatile("buffer_load_dwordx3 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r) : "memory");
    return v;
}
__device__ __forceinline__ void win_st64(__amdgpu_buffer_rsrc_t r, int off, double v) {
    asm volatile("buffer_store_dwordx2 %0, %1, %2, 0 offen" ::"v"(v), "v"(off), "s"(r) : "memory");
}
template <int N, bool RING, int KPW>
__device__ __forceinline__ void win_wait(WinBuf<KPW> &B) {  // vmcnt(N), B's registers pinned to it
    asm volatile("s_waitcnt vmcnt(%c0)" ::"n"(N) : "memory");
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(B.tv[k]));
#pragma unroll
    for (int u = 0; u < KPW; ++u) asm volatile("" : "+v"(B.sr[u]));
    if (RING) asm volatile("" : "+v"(B.rx));
}

// RING: ys is a ring of WIN_RING rows (row r in slot r mod WIN_RING; the setup
// checks that no row depends on one more than WIN_RING - 64 rows away), the
// window's input rows come from global memory (in, prefetched with the window's
// data) and its solution goes to global memory (out) as well as to the ring
template <bool UP, int WD, bool RING, int KPW>
__device__ __forceinline__ void win_sweep(int64_t len, int64_t w0, const int64_t *__restrict__ woff,
                                          const int32_t *__restrict__ rec, const double *__restrict__ tinv, double *ys,
                                          double *part, int lane, int q, const double *in = nullptr,
                                          double *out = nullptr, int64_t *lwo_lds = nullptr) {
    constexpr int R = RING ? 1 : WIN_OFFR, NL = win_loads<RING, KPW>();  // (ring: offsets in LDS)
    constexpr int64_t RM = WIN_RING - 1;
    const int64_t nw = (len + 63) >> 6;
    if (nw == 0) return;
    // the block's window stream offsets: registers (64 per register, picked by a
    // vector select and one readlane), or -- ring variant -- LDS (part + 576,
    // up to 1,024; a same-address read per window)
    // (the LDS variant too where they fit after the block: lwo_lds)
    WinOff<R> wo;
    int64_t *lwo = RING ? reinterpret_cast<int64_t *>(part + 576) : lwo_lds;
    const bool in_lds = RING || lwo_lds != nullptr;  // (uniform)
    if (in_lds) {
        for (int64_t t = threadIdx.x; t <= nw; t += 256) lwo[t] = woff[w0 + t];
        __syncthreads();
    } else {
#pragma unroll
        for (int j = 0; j < R; ++j) wo.r[j] = j * 64 + lane <= nw ? woff[w0 + j * 64 + lane] : 0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the offsets (ordinary loads) before the counted ones
    auto at = [&](int64_t w) -> int64_t { return in_lds ? sgpr64(lwo[w]) : wo.at(w); };
    const auto rin = win_rsrc(in, RING ? len * 8 : 0), rout = win_rsrc(out, RING ? len * 8 : 0);
    // (pls.ring_probe, ring variant, timing only -- results wrong: 2048 no stores,
    // 32768 no loads after the first two windows)
    const int probe = RING ? __builtin_amdgcn_readfirstlane(ring_probe) : 0;
    auto wi = [&](int64_t ww) { return UP ? nw - 1 - ww : ww; };
    // T^-1[lane][k], T^-1[lane][k + 1] (k even): both zero above (L) / below (U)
    // the diagonal -- those lanes read out of range
    auto toff = [&](int k) {
        return (UP ? k + 1 >= lane : k <= lane) ? (k >> 1) * 1024 + lane * 16 : 0x40000000;
    };
    auto sk = [&](int u) { return (u * WIN_NW + q) * 64 + lane; };  // this wave's u-th stream slot
    // every window's loads, NL in one fixed order (past the block: 0 bytes in range, no traffic)
    auto issue = [&](int64_t ww, WinBuf<KPW> &B) {
        if ((probe & 32768) && ww >= 2) return;
        const int64_t ok = ww < nw ? 1 : 0;
        const int64_t w = wi(ww < nw ? ww : 0);
        const int64_t s0 = at(w), s1 = at(w + 1);
        const auto rt = win_rsrc(tinv + (w0 + w) * 4096, ok * 32768);
        const auto rs = win_rsrc(rec + 3 * s0, ok * (s1 - s0) * 12);
#pragma unroll
        for (int u = 0; u < KPW; ++u) B.sr[u] = win_ld96(rs, sk(u) * 12);
#pragma unroll
        for (int j = 0; j < 8; ++j) B.tv[j] = win_ld128(rt, toff(16 * q + 2 * j));
        // (ring: wave 0 alone loads the input rows and stores the solution -- the
        // load instructions, not their lanes, are what a window costs)
        if (RING && q == 0) B.rx = win_ld64(rin, (int)(ok * (w * 64 + lane) * 8 + (1 - ok) * 0x40000000));
    };
    // one window, branch-free (a window past the block computes zeros into a dummy slot)
    auto compute = [&](int64_t ww, const WinBuf<KPW> &B) {
        const int64_t w = wi(ww < nw ? ww : 0);
        const int64_t r = w * 64 + lane;
        const bool act = ww < nw && r < len;
        double d[KPW];
#pragma unroll
        for (int u = 0; u < KPW; ++u) {
            const int32_t c = B.sr[u].z;
            d[u] = ys[RING ? (c & RM) : c];
        }
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < KPW; ++u) acc += __dmul_rn(__hiloint2double(B.sr[u].y, B.sr[u].x), d[u]);
        part[q * 64 + lane] = acc;
        double *rxs = part + 512;  // (ring: wave 0's input rows for every wave)
        if (RING && q == 0) rxs[lane] = B.rx;
        __syncthreads();
        const double rhs = RING ? rxs[lane] : ys[act ? r : 0];
        const double t = act ? rhs - (((part[lane] + part[64 + lane]) + part[128 + lane]) + part[192 + lane]) : 0.0;
        // t_k to every lane through the wave's own LDS slot (its own write: no
        // barrier; same-address reads broadcast) -- 32 v_readlane before
        double *tbq = part + 256 + q * 64;
        tbq[lane] = t;
        double out = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) out += __dmul_rn((k & 1) ? B.tv[k >> 1].y : B.tv[k >> 1].x, tbq[16 * q + k]);
        __syncthreads();  // every wave has read part[] (t) before it is overwritten
        part[q * 64 + lane] = out;
        __syncthreads();
        const double yr = ((part[lane] + part[64 + lane]) + part[128 + lane]) + part[192 + lane];
        if (RING) {
            // every wave stores the window (the same values): one counted store per
            // wave and window, issued after the window's loads
            ys[act ? (r & RM) : WIN_RING + lane] = yr;
            if (q == 0 && !(probe & 2048)) win_st64(rout, act ? (int)(r * 8) : 0x40000000, yr);
        } else {
            ys[act ? r : len + lane] = yr;  // every wave writes the same value (its own later reads see it)
        }
        __syncthreads();  // part[] free for the next window
        // (measured: double-buffering part[] to drop this barrier and the one above
        // was no faster -- 1,612 against 1,531 us per swelling N=160 chunk sweep)
    };
    if (WD == 3 && !RING) {
        // three windows of data in flight: the oldest window's loads are followed
        // by exactly 2 NL younger ones
        static_assert(2 * NL <= 63, "vmcnt counts 63");
        WinBuf<KPW> A, B, C;
        issue(0, A);
        issue(1, B);
        issue(2, C);
        for (int64_t ww = 0; ww < nw; ww += 3) {
            win_wait<2 * NL, false>(A);
            compute(ww, A);
            issue(ww + 3, A);
            win_wait<2 * NL, false>(B);
            compute(ww + 1, B);
            issue(ww + 4, B);
            win_wait<2 * NL, false>(C);
            compute(ww + 2, C);
            issue(ww + 5, C);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
    }
    // (ring: a window's store sits between its successor's loads and the next
    // issue; vector memory completes in issue order, so one more may be pending)
    // (ring: only wave 0 has the input load and the store; the other waves
    // count NL - 1 loads per window and no store)
    auto run = [&](auto w0) {
        constexpr bool S = RING && decltype(w0)::value;
        constexpr int NLq = RING && !S ? NL - 1 : NL, WT = S ? NL + 1 : NLq;
        WinBuf<KPW> A, B;
        issue(0, A);
        issue(1, B);
        if (S) win_wait<NLq, RING>(A);  // (no store yet between A and B)
        for (int64_t ww = 0; ww < nw; ww += 2) {  // two windows per trip: loads of window ww + 2 fly during ww + 1
            win_wait<WT, RING>(A);                // A's loads are older than B's (and a store)
            compute(ww, A);
            issue(ww + 2, A);
            win_wait<WT, RING>(B);
            compute(ww + 1, B);
            issue(ww + 3, B);
        }
    };
    if (RING && q == 0)
        run(std::integral_constant<bool, true>{});
    else
        run(std::integral_constant<bool, false>{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the prefetches past the block: nothing in range)
}

template <int WD, bool RING, int KL, int KU>
__global__ __launch_bounds__(256) void k_ilu_blocks_window(int64_t n, int64_t nblocks, const int64_t *__restrict__ bstart,
                                                           const int64_t *__restrict__ wstart,
                                                           const int64_t *__restrict__ Lwoff, const int32_t *__restrict__ Lrec,
                                                           const double *__restrict__ Ltinv,
                                                           const int64_t *__restrict__ Uwoff, const int32_t *__restrict__ Urec,
                                                           const double *__restrict__ Utinv, const double *x, double *y,
                                                           int tri, int lwo_ok) {
    // one dynamic LDS array: the partial sums (4 x 64), the waves' t (4 x 64), then the block solution
    extern __shared__ __attribute__((aligned(16))) double lds_win[];
    double *part = lds_win, *ys = lds_win + 512;
    const int64_t blk = nblocks - 1 - (int64_t)blockIdx.x;
    int64_t b0, len;
    block_range(blk, n, nblocks, bstart, b0, len);
    const int lane = threadIdx.x & 63;
    const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (v_readlane's lane is a scalar)
    if (RING)  // (padding entries read slot 0 with value 0: every slot finite)
        for (int64_t t = threadIdx.x; t < WIN_RING; t += 256) ys[1088 + t] = 0.0;  // (the ring: after rows, offsets)
    else
        for (int64_t t = threadIdx.x; t < len; t += 256) ys[t] = x[b0 + t];
    __syncthreads();
    // block bounds as scalars (buffer resources built from them must live in SGPRs)
    auto uni = [](int64_t v) {
        const int32_t lo = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)(uint64_t)v);
        const int32_t hi = __builtin_amdgcn_readfirstlane((int32_t)((uint64_t)v >> 32));
        return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
    };
    len = uni(len);
    const int64_t w0 = uni(wstart[blk]);
    if (RING) {
        // L: x -> y (global and the ring); U: y -> y in place, its input rows read
        // from global memory after every wave's L stores completed (win_sweep ends
        // with vmcnt(0); the barrier orders them before U's first loads)
        // (tri: 1 L, 2 U -- y already holds L's solution, the ring then only U's rows -- 3 both)
        // (ring layout: partial sums, t, wave 0's input rows (64), the window
        // offsets (1,024), then the ring)
        if (tri & 1) win_sweep<false, 2, true, KL>(len, w0, Lwoff, Lrec, Ltinv, ys + 1088, part, lane, q, x + b0, y + b0);
        __syncthreads();
        if (tri & 2) win_sweep<true, 2, true, KU>(len, w0, Uwoff, Urec, Utinv, ys + 1088, part, lane, q, y + b0, y + b0);
        return;
    }
    // (the window offsets after the block and its dummy slots, where the launch sized LDS for them)
    int64_t *lwo = lwo_ok ? reinterpret_cast<int64_t *>(ys + len + 64) : nullptr;
    win_sweep<false, WD, false, KL>(len, w0, Lwoff, Lrec, Ltinv, ys, part, lane, q, nullptr, nullptr, lwo);
    __syncthreads();  // (L's last offset reads before U's fill)
    win_sweep<true, WD, false, KU>(len, w0, Uwoff, Urec, Utinv, ys, part, lane, q, nullptr, nullptr, lwo);
    __syncthreads();
    for (int64_t t = threadIdx.x; t < len; t += 256) y[b0 + t] = ys[t];
}

int ilu_window_max_rows() { return 163840 / 8 - 512 - 64; }  // LDS: partial sums, t, the block, a dummy slot per lane
static_assert((163840 / 8 - 512 - 64 + 63) / 64 + 1 <= 64 * WIN_OFFR, "window offsets exceed WinOff's registers");
int ilu_window_ring_rows() { return WIN_RING; }
int64_t ilu_window_ring_max_rows() { return (int64_t)(64 * WIN_OFFR_RING - 1) * 64; }
static_assert(1600 + WIN_RING + 64 <= 163840 / 8, "the ring exceeds LDS");
static_assert(64 * WIN_OFFR_RING <= 1024, "the ring variant's window offsets exceed their LDS slots");
int ilu_window_stream_pad() { return 0; }
int ilu_window_max_entries() { return WIN_KP; }

template <int KL, int KU>
static void window_launch(int64_t n, int64_t nblocks, const int64_t *bstart, const int64_t *wstart,
                          const int64_t *Lwoff, const int32_t *Lrec, const double *Ltinv, const int64_t *Uwoff,
                          const int32_t *Urec, const double *Utinv, const double *x, double *y, int64_t max_len,
                          hipStream_t st, int depth, bool ring, int tri) {
    static bool configured = false;
    if (!configured) {
        for (const void *k : {(const void *)k_ilu_blocks_window<2, false, KL, KU>,
                              (const void *)k_ilu_blocks_window<3, false, KL, KU>,
                              (const void *)k_ilu_blocks_window<2, true, KL, KU>})
            (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)163840);
        configured = true;
    }
    if (ring) {  // (x may be y: a window's input rows are read before its solution is stored)
        const size_t bytes = (size_t)(1600 + WIN_RING + 64) * 8;
        k_ilu_blocks_window<2, true, KL, KU><<<(unsigned)nblocks, 256, bytes, st>>>(
            n, nblocks, bstart, wstart, Lwoff, Lrec, Ltinv, Uwoff, Urec, Utinv, x, y, tri, 0);
        return;
    }
    size_t bytes = (size_t)(512 + std::max<int64_t>(max_len, 1) + 64) * 8;  // + a dummy slot per lane
    const size_t obytes = (size_t)((std::max<int64_t>(max_len, 1) + 63) / 64 + 1) * 8;  // the window offsets
    const int lwo_ok = bytes + obytes <= 163840 ? 1 : 0;
    if (lwo_ok) bytes += obytes;
    if (depth == 3)
        k_ilu_blocks_window<3, false, KL, KU><<<(unsigned)nblocks, 256, bytes, st>>>(
            n, nblocks, bstart, wstart, Lwoff, Lrec, Ltinv, Uwoff, Urec, Utinv, x, y, 3, lwo_ok);
    else
        k_ilu_blocks_window<2, false, KL, KU><<<(unsigned)nblocks, 256, bytes, st>>>(
            n, nblocks, bstart, wstart, Lwoff, Lrec, Ltinv, Uwoff, Urec, Utinv, x, y, 3, lwo_ok);
}
int window_records(int max_entries) {  // stream records per wave and window: 4, 6 or 8
    return max_entries <= 4 * WIN_NW ? 4 : max_entries <= 6 * WIN_NW ? 6 : WIN_KPW;
}
template <int KL>
static void window_launch_u(int ku, int64_t n, int64_t nblocks, const int64_t *bstart, const int64_t *wstart,
                            const int64_t *Lwoff, const int32_t *Lrec, const double *Ltinv, const int64_t *Uwoff,
                            const int32_t *Urec, const double *Utinv, const double *x, double *y, int64_t max_len,
                            hipStream_t st, int depth, bool ring, int tri) {
    if (ku == 4)
        window_launch<KL, 4>(n, nblocks, bstart, wstart, Lwoff, Lrec, Ltinv, Uwoff, Urec, Utinv, x, y, max_len, st,
                             depth, ring, tri);
    else if (ku == 6)
        window_launch<KL, 6>(n, nblocks, bstart, wstart, Lwoff, Lrec, Ltinv, Uwoff, Urec, Utinv, x, y, max_len, st,
                             depth, ring, tri);
    else
        window_launch<KL, WIN_KPW>(n, nblocks, bstart, wstart, Lwoff, Lrec, Ltinv, Uwoff, Urec, Utinv, x, y, max_len,
                                   st, depth, ring, tri);
}
void launch_ilu_blocks_window(int64_t n, int64_t nblocks, const int64_t *bstart, const int64_t *wstart,
                              const int64_t *Lwoff, const int32_t *Lrec, const double *Ltinv, const int64_t *Uwoff,
                              const int32_t *Urec, const double *Utinv, const double *x, double *y, int64_t max_len,
                              hipStream_t st, int depth, bool ring, int tri, int max_entries_L, int max_entries_U) {
    const int kl = window_records(max_entries_L), ku = window_records(max_entries_U);
    if (kl == 4)
        window_launch_u<4>(ku, n, nblocks, bstart, wstart, Lwoff, Lrec, Ltinv, Uwoff, Urec, Utinv, x, y, max_len, st,
                           depth, ring, tri);
    else if (kl == 6)
        window_launch_u<6>(ku, n, nblocks, bstart, wstart, Lwoff, Lrec, Ltinv, Uwoff, Urec, Utinv, x, y, max_len, st,
                           depth, ring, tri);
    else
        window_launch_u<WIN_KPW>(ku, n, nblocks, bstart, wstart, Lwoff, Lrec, Ltinv, Uwoff, Urec, Utinv, x, y, max_len,
                                 st, depth, ring, tri);
}

// ======================================================= super-window sweep ==
// Triangular sweeps of blocks too long for LDS (whole FE blocks: ~47k rows at
// 3-D N=12, 353k at N=24, whose level DAGs are ~1,440 / ~2,985 levels deep).
// Rows are cut into windows of 64 (lane = row) and consecutive windows into
// super-windows (build_swin_tri): per super-window, in processing order,
//   1. all waves stage the super-window's packed window inverses and near
//      streams into LDS, and every row's input minus its far terms (entries
//      before the super-window, read from the block solution in global
//      memory -- final since earlier super-windows) goes to LDS;
//   2. one wave walks the windows: t = input - near terms (LDS gathers),
//      y = T_w^-1 t (a 64 x 64 triangular GEMV from LDS, t broadcast with
//      v_readlane), y to LDS -- no barrier between windows (a wave's LDS
//      accesses complete in order);
//   3. the super-window's y to global memory.
// The dependent chain is the windows' GEMVs (len / 64 per triangle) instead of
// the levels; no global load sits on it.  L: input x, output y; U: in place on
// y.  Sums: far terms, near terms (stream order), then the window inverse --
// the explicit inverses reassociate the substitution's sums (<= 1e-12 against
// the level-order sweeps, tests/test_gpu_sweeps.py).
static constexpr int SWIN_TPB = 256, SWIN_TRI = 2080;

// global -> LDS copies of the staged streams: 8 x 16 bytes in flight per thread
__device__ __forceinline__ void swin_copy(const double *__restrict__ src, double *dst, int64_t n, int tid) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    const bool al = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
    if (!al) {
        for (int64_t k = tid; k < n; k += SWIN_TPB) dst[k] = src[k];
        return;
    }
    const int64_t n2 = n >> 1;
    const d2 *s2 = reinterpret_cast<const d2 *>(src);
    d2 *t2 = reinterpret_cast<d2 *>(dst);
    for (int64_t k0 = 0; k0 < n2; k0 += 8 * SWIN_TPB) {
        d2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t k = k0 + u * SWIN_TPB + tid;
            v[u] = k < n2 ? s2[k] : d2{0.0, 0.0};
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t k = k0 + u * SWIN_TPB + tid;
            if (k < n2) t2[k] = v[u];
        }
    }
    if ((n & 1) && tid == 0) dst[n - 1] = src[n - 1];
}
__device__ __forceinline__ void swin_copy32(const int32_t *__restrict__ src, int32_t *dst, int64_t n, int tid) {
    for (int64_t k0 = 0; k0 < n; k0 += 8 * SWIN_TPB) {
        int32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t k = k0 + u * SWIN_TPB + tid;
            v[u] = k < n ? src[k] : 0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t k = k0 + u * SWIN_TPB + tid;
            if (k < n) dst[k] = v[u];
        }
    }
}

template <bool UP>
__device__ __forceinline__ void swin_sweep(int64_t len, int64_t bs0, int64_t bs1, const int64_t *__restrict__ sw,
                                           const int64_t *__restrict__ wnear, const int32_t *__restrict__ ncol,
                                           const double *__restrict__ nval, const int64_t *__restrict__ wfar,
                                           const int32_t *__restrict__ fcol, const double *__restrict__ fval,
                                           const double *__restrict__ tinv, int64_t wfirst, const double *in,
                                           double *out, double *lds) {
    double *ys = lds;            // the super-window's rows (<= 512)
    double *tb = lds + 512;      // the window's t, broadcast
    double *ts = lds + 576;      // staged inverses, then near values
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int64_t s = bs0; s < bs1; ++s) {
        const int64_t w0 = sw[4 * s], nwn = sw[4 * s + 1], r0 = sw[4 * s + 2], r1 = sw[4 * s + 3];
        // 1. stage: inverses (nwn * 2080 doubles), near values and columns
        const int64_t nt = nwn * SWIN_TRI, e0 = wnear[w0], ne = wnear[w0 + nwn] - e0;
        double *nv = ts + nt;
        int32_t *nc = reinterpret_cast<int32_t *>(nv + ne);
        // (eight 16-byte loads in flight per thread, then their LDS stores: the copies
        // are latency-bound, one round trip per round)
        // (pls.ring_probe bits 256 / 512 / 1024: no staging / far terms / window chain --
        // timing diagnostics, results wrong)
        const int probe = ring_probe;
        if (!(probe & 256)) {
            swin_copy(reinterpret_cast<const double *>(tinv) + w0 * SWIN_TRI, ts, nt, tid);
            swin_copy(nval + e0, nv, ne, tid);
            swin_copy32(ncol + e0, nc, ne, tid);
        }
        // far terms: one row per thread (64-row slices: [k][lane] streams), eight gathers in flight
        for (int64_t r = r0 + tid; r < r1; r += SWIN_TPB) {
            const int64_t w = wfirst + (r >> 6), l = r & 63;
            const int64_t f0 = wfar[w], K = (probe & 512) ? 0 : (wfar[w + 1] - f0) >> 6;
            double acc = 0.0;
            const double xin = in[r];
            for (int64_t k = 0; k < K; k += 8) {
                int32_t cc[8];
                double vv[8], yy[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int64_t kk = k + u < K ? k + u : K - 1;  // (clamped: the value is zeroed below)
                    cc[u] = fcol[f0 + kk * 64 + l];
                    vv[u] = fval[f0 + kk * 64 + l];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) yy[u] = out[cc[u]];
#pragma unroll
                for (int u = 0; u < 8; ++u) acc += __dmul_rn(k + u < K ? vv[u] : 0.0, yy[u]);
            }
            ys[r - r0] = xin - acc;
        }
        __syncthreads();
        // 2. the windows, one wave
        if (wave == 0 && !(probe & 1024)) {
            for (int64_t j0 = 0; j0 < nwn; ++j0) {
                const int64_t j = UP ? nwn - 1 - j0 : j0;
                const int64_t w = w0 + j, wr = (w - wfirst) * 64;  // window's first row (block-local)
                const bool act = wr + lane < len;
                const int64_t q0 = wnear[w] - e0, K = (wnear[w + 1] - wnear[w]) >> 6;
                // near terms, eight at a time: their column / value reads, then the
                // eight y gathers, all issued before the first is used (branch-free:
                // padding and the tail read entry 0 with value 0)
                double acc = 0.0;
                for (int64_t k0 = 0; k0 < K; k0 += 8) {
                    int32_t cc[8];
                    double vv[8], yy[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int64_t q = q0 + (k0 + u < K ? k0 + u : 0) * 64 + lane;
                        cc[u] = nc[q];
                        vv[u] = k0 + u < K ? nv[q] : 0.0;
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) yy[u] = ys[cc[u]];
#pragma unroll
                    for (int u = 0; u < 8; ++u) acc += __dmul_rn(vv[u], yy[u]);
                }
                const double t = act ? ys[wr - r0 + lane] - acc : 0.0;
                tb[lane] = t;  // broadcast through LDS (one wave: in order, no barrier)
                const double *T = ts + j * SWIN_TRI;
                // y = T^-1 t: 16 columns per step, their LDS reads (T column entries and
                // the broadcast t_k) issued together; four partial sums (k mod 4) added
                // in a fixed order
                double ya[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int k0 = 0; k0 < 64; k0 += 16) {
                    double a[16], tk[16];
#pragma unroll
                    for (int u = 0; u < 16; ++u) {
                        const int k = k0 + u;
                        const bool nz = UP ? lane <= k : lane >= k;
                        const int off = UP ? k * (k + 1) / 2 + lane : 64 * k - k * (k - 1) / 2 + (lane - k);
                        a[u] = T[nz ? off : 0];
                        tk[u] = tb[k];
                    }
#pragma unroll
                    for (int u = 0; u < 16; ++u) {
                        const int k = k0 + u;
                        const bool nz = UP ? lane <= k : lane >= k;
                        ya[u & 3] = __fma_rn(nz ? a[u] : 0.0, tk[u], ya[u & 3]);
                    }
                }
                const double y = (ya[0] + ya[1]) + (ya[2] + ya[3]);
                if (act) ys[wr - r0 + lane] = y;
            }
        }
        __syncthreads();
        // 3. the super-window's solution to global memory (far terms of later super-windows read it)
        for (int64_t r = r0 + tid; r < r1; r += SWIN_TPB) out[r] = ys[r - r0];
        __syncthreads();
    }
}

__global__ __launch_bounds__(SWIN_TPB) void k_ilu_blocks_swin(
    int64_t n, int64_t nblocks, const int64_t *__restrict__ bstart, const int64_t *__restrict__ wstart,
    const int64_t *__restrict__ Lbsw, const int64_t *__restrict__ Lsw, const int64_t *__restrict__ Lwnear,
    const int32_t *__restrict__ Lncol, const double *__restrict__ Lnval, const int64_t *__restrict__ Lwfar,
    const int32_t *__restrict__ Lfcol, const double *__restrict__ Lfval, const double *__restrict__ Ltinv,
    const int64_t *__restrict__ Ubsw, const int64_t *__restrict__ Usw, const int64_t *__restrict__ Uwnear,
    const int32_t *__restrict__ Uncol, const double *__restrict__ Unval, const int64_t *__restrict__ Uwfar,
    const int32_t *__restrict__ Ufcol, const double *__restrict__ Ufval, const double *__restrict__ Utinv,
    const double *x, double *y) {
    extern __shared__ __attribute__((aligned(16))) double lds_sw[];
    const int64_t blk = nblocks - 1 - (int64_t)blockIdx.x;
    int64_t b0, len;
    block_range(blk, n, nblocks, bstart, b0, len);
    const int64_t wf = wstart[blk];
    swin_sweep<false>(len, Lbsw[blk], Lbsw[blk + 1], Lsw, Lwnear, Lncol, Lnval, Lwfar, Lfcol + 0, Lfval, Ltinv, wf,
                      x + b0, y + b0, lds_sw);
    swin_sweep<true>(len, Ubsw[blk], Ubsw[blk + 1], Usw, Uwnear, Uncol, Unval, Uwfar, Ufcol, Ufval, Utinv, wf, y + b0,
                     y + b0, lds_sw);
}

int ilu_swin_lds_budget() { return 163840 - 576 * 8 - 1024; }

void launch_ilu_blocks_swin(int64_t n, int64_t nblocks, const int64_t *bstart, const int64_t *wstart,
                            const int64_t *Lbsw, const int64_t *Lsw, const int64_t *Lwnear, const int32_t *Lncol,
                            const double *Lnval, const int64_t *Lwfar, const int32_t *Lfcol, const double *Lfval,
                            const double *Ltinv, const int64_t *Ubsw, const int64_t *Usw, const int64_t *Uwnear,
                            const int32_t *Uncol, const double *Unval, const int64_t *Uwfar, const int32_t *Ufcol,
                            const double *Ufval, const double *Utinv, const double *x, double *y, int64_t lds_bytes,
                            hipStream_t st) {
    static bool configured = false;
    if (!configured) {
        (void)hipFuncSetAttribute((const void *)k_ilu_blocks_swin, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)163840);
        configured = true;
    }
    k_ilu_blocks_swin<<<(unsigned)nblocks, SWIN_TPB, (size_t)lds_bytes, st>>>(
        n, nblocks, bstart, wstart, Lbsw, Lsw, Lwnear, Lncol, Lnval, Lwfar, Lfcol, Lfval, Ltinv, Ubsw, Usw, Uwnear,
        Uncol, Unval, Uwfar, Ufcol, Ufval, Utinv, x, y);
}

// =========================================================== distribution ====
// flag[c] = 1 for every column c (relative to the column space) of the matrix
// that this rank does not own (own[c] < 0)
__global__ __launch_bounds__(TPB) void k_flag_ghosts(int64_t nnz, const int32_t *ci, const int32_t *own, uint8_t *flag) {
    for (int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x; k < nnz; k += (int64_t)gridDim.x * TPB) {
        const int32_t c = ci[k];
        if (own[c] < 0) flag[c] = 1;
    }
}
__global__ __launch_bounds__(TPB) void k_remap_cols(int64_t nnz, int32_t *ci, const int32_t *gmap) {
    for (int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x; k < nnz; k += (int64_t)gridDim.x * TPB)
        ci[k] = gmap[ci[k]];
}
__global__ __launch_bounds__(TPB) void k_pack(int64_t m, const int32_t *idx, const double *x, double *buf) {
    const int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (k < m) buf[k] = x[idx[k]];
}
void launch_flag_ghosts(int64_t nnz, const int32_t *ci, const int32_t *own, uint8_t *flag, hipStream_t st) {
    if (nnz > 0) k_flag_ghosts<<<stream_grid(nnz), TPB, 0, st>>>(nnz, ci, own, flag);
}
void launch_remap_cols(int64_t nnz, int32_t *ci, const int32_t *gmap, hipStream_t st) {
    if (nnz > 0) k_remap_cols<<<stream_grid(nnz), TPB, 0, st>>>(nnz, ci, gmap);
}
// Remapped rows are sorted runs (owned columns in order, ghosts per owner and
// field in order) -> restore ascending columns; one thread per row, insertion
// sort (setup only; every consumer -- window extraction, diagonal search, ILU
// pattern matching -- binary-searches sorted rows).
__global__ __launch_bounds__(TPB) void k_sort_rows(int64_t n, const int64_t *rp, int32_t *ci, double *val) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    const int64_t s = rp[i], e = rp[i + 1];
    for (int64_t k = s + 1; k < e; ++k) {
        const int32_t c = ci[k];
        const double v = val[k];
        int64_t j = k - 1;
        while (j >= s && ci[j] > c) {
            ci[j + 1] = ci[j];
            val[j + 1] = val[j];
            --j;
        }
        ci[j + 1] = c;
        val[j + 1] = v;
    }
}
void launch_sort_rows(int64_t n, const int64_t *rp, int32_t *ci, double *val, hipStream_t st) {
    if (n > 0) k_sort_rows<<<grid_for(n, TPB), TPB, 0, st>>>(n, rp, ci, val);
}
__global__ __launch_bounds__(TPB) void k_unpack(int64_t m, const int32_t *idx, const double *buf, double *x) {
    const int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (k < m) x[idx[k]] = buf[k];
}
void launch_unpack(int64_t m, const int32_t *idx, const double *buf, double *x, hipStream_t st) {
    if (m > 0) k_unpack<<<grid_for(m, TPB), TPB, 0, st>>>(m, idx, buf, x);
}
void launch_pack(int64_t m, const int32_t *idx, const double *x, double *buf, hipStream_t st) {
    if (m > 0) k_pack<<<grid_for(m, TPB), TPB, 0, st>>>(m, idx, x, buf);
}

}  // namespace pls
