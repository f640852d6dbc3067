// band.hip -- exact LU (PCLU) of large banded field blocks.
//
// The reference's exact option set factors every block with MUMPS
// (petsc-options-exact:11-35) and the inexact set factors the Schur block of
// the fp fieldsplit with it (petsc-options-inexact:98-106).  Blocks too large
// for the dense inverse (dense.hip) but with a bounded band -- the field blocks
// of a bandwidth-reduced FE ordering, and the selfp Schur matrix -- are factored
// here as block-banded matrices of 64 x 64 tiles without pivoting (like the
// natural-ordering factorization of these diagonally dominant blocks): fill
// stays inside the band, so the factorization is exact.
//
// Storage: tile row I holds tiles J = I - bl .. I + bu at T[(I W + J - I + bl)
// * 4096] (row-major 64 x 64, W = bl + bu + 1); rows/columns past n are identity
// padding.  After the factorization the strictly lower tiles hold L, the upper
// tiles U and the diagonal tiles L\U; Dl[I] = L_II^-1 and Du[I] = U_II^-1
// (64 x 64 each) serve the sweeps.
//
// Factorization (right-looking, one tile column per step K): k_band_diag
// factors T_KK in LDS and inverts its triangles; k_band_panels forms
// L_IK = A_IK Du_K and U_KJ = Dl_K A_KJ; k_band_update applies
// A_IJ -= L_IK U_KJ to the bl x bu trailing window.  ~2 n kl ku flops, all on
// 64 x 64 LDS tiles.
//
// Sweeps: one launch per triangle.  Workgroups take tile rows from a ticket
// counter, so every row a workgroup waits on belongs to a workgroup that is
// already running (no dispatch-order or residency assumption); each
// accumulates its band tiles against the y blocks as they are published, the
// nearest block last, and publishes y_I = Dinv_I r_I.  Hand-off (the producer
// may sit on another XCD; cdna_hip_programming.md Guideline 16, R2): y_I is
// published as tagged 8-byte granules (sc1 stores) that a consumer wave
// re-reads (sc1 loads, bounded spin) until every tag carries this sweep's
// epoch -- no flag, fence or drain.  The sums run in a fixed order, so the
// result does not depend on timing.  HBM traffic is the band once per sweep;
// the critical path is one hop per 64 rows.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace pls {

static constexpr int BT = 64;     // tile size
static constexpr int BTPB = 256;  // threads per workgroup
static constexpr int64_t TILE = BT * BT;

typedef __attribute__((address_space(1))) uint64_t gu64;

// ------------------------------------------------------------------ build --
// identity on the padding diagonal (T zeroed first), then the CSR rows
__global__ __launch_bounds__(256) void k_band_pad(int64_t n, int64_t nb, int64_t W, int64_t bl, double *T) {
    const int64_t i = n + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nb * BT) return;
    const int64_t I = i / BT, r = i % BT;
    T[(I * W + bl) * TILE + r * BT + r] = 1.0;
}
__global__ __launch_bounds__(256) void k_band_scatter(int64_t n, int64_t W, int64_t bl, const int64_t *rp,
                                                      const int32_t *ci, const double *val, double *T) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const int64_t I = i / BT, r = i % BT;
    for (int64_t k = rp[i] + (threadIdx.x & 63); k < rp[i + 1]; k += 64) {
        const int64_t j = ci[k], J = j / BT;
        T[(I * W + (J - I + bl)) * TILE + r * BT + (j % BT)] = val[k];
    }
}
void launch_band_from_csr(int64_t n, int64_t nb, int64_t bl, int64_t bu, const int64_t *rp, const int32_t *ci,
                          const double *val, double *T, hipStream_t st) {
    const int64_t W = bl + bu + 1;
    (void)hipMemsetAsync(T, 0, sizeof(double) * (size_t)(nb * W * TILE), st);
    if (nb * BT > n) k_band_pad<<<(unsigned)((nb * BT - n + 255) / 256), 256, 0, st>>>(n, nb, W, bl, T);
    if (n > 0) k_band_scatter<<<(unsigned)((n + 3) / 4), 256, 0, st>>>(n, W, bl, rp, ci, val, T);
}

// ----------------------------------------------------------- factorization --
#pragma clang fp contract(off)
// LU of the diagonal tile in LDS (no pivoting), written back as L\U; Dl = L^-1
// (unit lower), Du = U^-1.  fail |= 1 on a zero pivot.
__global__ __launch_bounds__(BTPB) void k_band_diag(int64_t W, int64_t bl, int64_t K, double *T, double *Dl,
                                                    double *Du, int32_t *fail) {
    __shared__ double a[BT][BT + 1];
    __shared__ double li[BT][BT + 1];
    __shared__ double ui[BT][BT + 1];
    double *src = T + (K * W + bl) * TILE;
    for (int t = threadIdx.x; t < BT * BT; t += BTPB) {
        const int i = t / BT, j = t % BT;
        a[i][j] = src[t];
        li[i][j] = ui[i][j] = (i == j) ? 1.0 : 0.0;
    }
    __syncthreads();
    // forward elimination of [A | I]: A -> L\U, I -> L^-1 (the same row
    // operations); every thread updates 32 entries per step
    for (int p = 0; p < BT; ++p) {
        const double piv = a[p][p];
        if (piv == 0.0) {
            if (threadIdx.x == 0) atomicOr(fail, 1);
            return;  // uniform across the workgroup (every thread read the same pivot)
        }
        if (p == BT - 1) break;
        __syncthreads();
        if (threadIdx.x > p && threadIdx.x < BT) a[threadIdx.x][p] = a[threadIdx.x][p] / piv;  // l_ip
        __syncthreads();
        for (int t = threadIdx.x; t < 2 * BT * BT; t += BTPB) {
            const int i = t / (2 * BT), j = t % (2 * BT);
            if (i <= p) continue;
            if (j < BT) {
                if (j > p) a[i][j] = a[i][j] - a[i][p] * a[p][j];
            } else if (j - BT <= p) {
                li[i][j - BT] = li[i][j - BT] - a[i][p] * li[p][j - BT];
            }
        }
        __syncthreads();
    }
    // backward elimination of [U | I] -> U^-1 (U itself stays in a)
    for (int p = BT - 1; p >= 0; --p) {
        if (threadIdx.x >= p && threadIdx.x < BT) ui[p][threadIdx.x] = ui[p][threadIdx.x] / a[p][p];
        __syncthreads();
        for (int t = threadIdx.x; t < p * BT; t += BTPB) {
            const int i = t / BT, j = t % BT;
            if (j >= p) ui[i][j] = ui[i][j] - a[i][p] * ui[p][j];
        }
        __syncthreads();
    }
    for (int t = threadIdx.x; t < BT * BT; t += BTPB) {
        const int i = t / BT, j = t % BT;
        src[t] = a[i][j];
        Dl[K * TILE + t] = li[i][j];
        Du[K * TILE + t] = ui[i][j];
    }
}
#pragma clang fp contract(on)

// acc = A B for 64 x 64 tiles staged in LDS (A transposed so its reads
// broadcast), 4 x 4 outputs per thread.
__device__ __forceinline__ void band_tile_mm(const double *A, const double *B, double (*at)[BT + 1],
                                             double (*b)[BT + 1], double acc[4][4]) {
    for (int t = threadIdx.x; t < BT * BT; t += BTPB) {
        const int r = t / BT, cc = t % BT;
        at[cc][r] = A[t];
        b[r][cc] = B[t];
    }
    __syncthreads();
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[r][q] = 0.0;
    for (int kk = 0; kk < BT; ++kk) {
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

// Panels of step K: blockIdx.x < bl: L_IK = A_IK Du_K (I = K + 1 + x);
// otherwise U_KJ = Dl_K A_KJ (J = K + 1 + x - bl).
__global__ __launch_bounds__(BTPB) void k_band_panels(int64_t nb, int64_t W, int64_t bl, int64_t K, double *T,
                                                      const double *Dl, const double *Du) {
    __shared__ double at[BT][BT + 1];
    __shared__ double b[BT][BT + 1];
    double acc[4][4];
    double *C;
    if ((int64_t)blockIdx.x < bl) {
        const int64_t I = K + 1 + blockIdx.x;
        if (I >= nb) return;
        C = T + (I * W + (K - I + bl)) * TILE;
        band_tile_mm(C, Du + K * TILE, at, b, acc);
    } else {
        const int64_t J = K + 1 + (blockIdx.x - bl);
        if (J >= nb) return;
        C = T + (K * W + (J - K + bl)) * TILE;
        band_tile_mm(Dl + K * TILE, C, at, b, acc);
    }
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) C[(ty + 16 * r) * BT + tx + 16 * q] = acc[r][q];
}

// Trailing update of step K: A_IJ -= L_IK U_KJ, I = K + 1 + y, J = K + 1 + x.
__global__ __launch_bounds__(BTPB) void k_band_update(int64_t nb, int64_t W, int64_t bl, int64_t K, double *T) {
    __shared__ double at[BT][BT + 1];
    __shared__ double b[BT][BT + 1];
    const int64_t I = K + 1 + blockIdx.y, J = K + 1 + blockIdx.x;
    if (I >= nb || J >= nb) return;
    double acc[4][4];
    band_tile_mm(T + (I * W + (K - I + bl)) * TILE, T + (K * W + (J - K + bl)) * TILE, at, b, acc);
    double *C = T + (I * W + (J - I + bl)) * TILE;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double *c = C + (ty + 16 * r) * BT + tx + 16 * q;
            *c = *c - acc[r][q];
        }
}

void launch_band_factor(int64_t nb, int64_t bl, int64_t bu, double *T, double *Dl, double *Du, int32_t *fail,
                        hipStream_t st) {
    const int64_t W = bl + bu + 1;
    for (int64_t K = 0; K < nb; ++K) {
        k_band_diag<<<1, BTPB, 0, st>>>(W, bl, K, T, Dl, Du, fail);
        const int64_t rest = nb - 1 - K;
        const int64_t pl = bl < rest ? bl : rest, pu = bu < rest ? bu : rest;
        if (pl + pu == 0) continue;
        k_band_panels<<<(unsigned)(bl + pu), BTPB, 0, st>>>(nb, W, bl, K, T, Dl, Du);
        if (pl > 0 && pu > 0) k_band_update<<<dim3((unsigned)pu, (unsigned)pl), BTPB, 0, st>>>(nb, W, bl, K, T);
    }
}

// ------------------------------------------------------------------ sweeps --
typedef double bd_d2 __attribute__((ext_vector_type(2)));

// One triangle (upper = 0: forward with L and Dl; 1: backward with U and Du):
// y_I = Dinv_I (b_I - sum_J T_IJ y_J).  Thread t owns row t / 4 and columns
// 16 (t % 4) .. +16 of every tile; b and y have n entries (padding rows are 0
// and never stored); b must not alias y.
// Hand-off (Guideline 16 R2, the data is the flag): y_I is published as 128
// 8-byte granules {epoch, 32 bits of y} in G (tile row I: G[128 I + 2 r + h],
// h = 0 low / 1 high half of row r), each written by ONE sc1 store; a
// consumer wave re-reads a tile row's 128 granules with sc1 loads until every
// tag equals this sweep's epoch (bounded spin), then stages y_J in LDS.  No
// flag, no fence, no drain.  The caller passes a fresh epoch (never 0; G
// starts zeroed) and the ticket count of all earlier sweeps as ticket_base.
__global__ __launch_bounds__(BTPB) void k_band_sweep(int64_t n, int64_t nb, int64_t bl, int64_t bu,
                                                     const double *__restrict__ T, const double *__restrict__ Dinv,
                                                     const double *__restrict__ b, double *__restrict__ y,
                                                     uint64_t *G, uint64_t *ticket, uint64_t ticket_base,
                                                     uint32_t epoch, int upper, int32_t *fail) {
    __shared__ int64_t sI;
    __shared__ double ys[BT];
    __shared__ double rs[BT];
    if (threadIdx.x == 0) sI = (int64_t)(atomicAdd((unsigned long long *)ticket, 1ull) - ticket_base);
    __syncthreads();
    const int64_t tk = sI;
    if (tk < 0 || tk >= nb) return;  // uniform
    const int64_t I = upper ? nb - 1 - tk : tk;
    const int64_t W = bl + bu + 1;
    const int row = threadIdx.x >> 2, part = threadIdx.x & 3;
    gu64 *gg = (gu64 *)G;
    const int64_t gi = I * BT + row;
    // everything off the dependency chain is loaded first
    const double bi = (part == 0 && gi < n) ? b[gi] : 0.0;
    bd_d2 dm[8];
    {
        const bd_d2 *dt = reinterpret_cast<const bd_d2 *>(Dinv + I * TILE + row * BT + part * 16);
#pragma unroll
        for (int u = 0; u < 8; ++u) dm[u] = dt[u];
    }
    int64_t J0, nJ;  // tiles to accumulate, farthest first
    if (upper) {
        J0 = (I + bu < nb - 1) ? I + bu : nb - 1;
        nJ = J0 - I;
    } else {
        J0 = (I - bl > 0) ? I - bl : 0;
        nJ = I - J0;
    }
    double acc = 0.0;
    for (int64_t s = 0; s < nJ; ++s) {
        const int64_t J = upper ? J0 - s : J0 + s;
        const bd_d2 *tile =
            reinterpret_cast<const bd_d2 *>(T + (I * W + (J - I + bl)) * TILE + row * BT + part * 16);
        bd_d2 m[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) m[u] = __builtin_nontemporal_load(tile + u);
        if (threadIdx.x < 64) {  // wave 0 sweeps tile row J's granules
            const int l = threadIdx.x;
            gu64 *g = gg + J * 128 + 2 * l;
            uint64_t lo = 0, hi = 0;
            for (int64_t spins = 0;; ++spins) {
                lo = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                hi = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const bool ok = (uint32_t)(lo >> 32) == epoch && (uint32_t)(hi >> 32) == epoch;
                if (__all(ok)) break;
                if (spins > (1ll << 26)) {  // never expected: report instead of hanging the queue
                    if (l == 0) atomicOr(fail, 2);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            ys[l] = __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            acc += m[u].x * ys[part * 16 + 2 * u];
            acc += m[u].y * ys[part * 16 + 2 * u + 1];
        }
        __syncthreads();  // ys is refilled for the next tile
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (part == 0) rs[row] = bi - acc;
    __syncthreads();
    double z = 0.0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        z += dm[u].x * rs[part * 16 + 2 * u];
        z += dm[u].y * rs[part * 16 + 2 * u + 1];
    }
    z += __shfl_xor(z, 1);
    z += __shfl_xor(z, 2);
    if (part == 0) {
        const uint64_t bits = gi < n ? (uint64_t)__double_as_longlong(z) : 0ull;  // padding rows publish 0
        const uint64_t tag = (uint64_t)epoch << 32;
        __hip_atomic_store(gg + I * 128 + 2 * row, tag | (bits & 0xffffffffull), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gg + I * 128 + 2 * row + 1, tag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (gi < n) y[gi] = z;
    }
}

void launch_band_sweep(int64_t n, int64_t nb, int64_t bl, int64_t bu, const double *T, const double *Dinv,
                       const double *b, double *y, uint64_t *G, uint64_t *ticket, uint64_t ticket_base,
                       uint32_t epoch, int upper, int32_t *fail, hipStream_t st) {
    if (nb > 0)
        k_band_sweep<<<(unsigned)nb, BTPB, 0, st>>>(n, nb, bl, bu, T, Dinv, b, y, G, ticket, ticket_base, epoch,
                                                   upper, fail);
}

}  // namespace pls
