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
// may sit on another XCD; cdna_hip_programming.md Guideline 16, R1): y stored
// write-through (global sc1), every storing wave drains (vmcnt(0)), workgroup
// barrier, one lane stores the tile row's flag (sc1); the consumer polls the
// flag from one lane (sc1, bounded spin), joins a barrier, and reads y with
// global sc1 loads only.  The sums run in a fixed order, so the result does
// not depend on timing.  HBM traffic is the band once per sweep; the critical
// path is one hop per 64 rows.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace pls {

static constexpr int BT = 64;     // tile size
static constexpr int BTPB = 256;  // threads per workgroup
static constexpr int64_t TILE = BT * BT;

typedef __attribute__((address_space(1))) double gf64;
typedef __attribute__((address_space(1))) int32_t gi32;

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
    for (int t = threadIdx.x; t < BT * BT; t += BTPB) a[t / BT][t % BT] = src[t];
    __syncthreads();
    for (int p = 0; p < BT; ++p) {
        const double piv = a[p][p];
        if (piv == 0.0) {
            if (threadIdx.x == 0) atomicOr(fail, 1);
            return;  // uniform across the workgroup (every thread read the same pivot)
        }
        if (p == BT - 1) break;
        __syncthreads();
        // multipliers l_ip = a_ip / piv, then the trailing update
        if (threadIdx.x > p && threadIdx.x < BT) a[threadIdx.x][p] = a[threadIdx.x][p] / piv;
        __syncthreads();
        for (int t = threadIdx.x; t < BT * BT; t += BTPB) {
            const int i = t / BT, j = t % BT;
            if (i > p && j > p) a[i][j] = a[i][j] - a[i][p] * a[p][j];
        }
        __syncthreads();
    }
    // triangular inverses, one column per thread: L^-1 e_j by forward and
    // U^-1 e_j by backward substitution
    if (threadIdx.x < BT) {
        const int j = threadIdx.x;
        for (int i = 0; i < BT; ++i) {
            double s = (i == j) ? 1.0 : 0.0;
            for (int k = j; k < i; ++k) s = s - a[i][k] * li[k][j];
            li[i][j] = (i < j) ? 0.0 : s;
        }
    } else if (threadIdx.x < 2 * BT) {
        const int j = threadIdx.x - BT;
        for (int i = BT - 1; i >= 0; --i) {
            double s = (i == j) ? 1.0 : 0.0;
            for (int k = i + 1; k <= j; ++k) s = s - a[i][k] * ui[k][j];
            ui[i][j] = (i > j) ? 0.0 : s / a[i][i];
        }
    }
    __syncthreads();
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
// and never stored); b must not alias y.  flags[I] == epoch publishes y_I;
// the caller passes a fresh epoch (never 0) and the ticket count of all
// earlier sweeps on this counter as ticket_base.
__global__ __launch_bounds__(BTPB) void k_band_sweep(int64_t n, int64_t nb, int64_t bl, int64_t bu,
                                                     const double *__restrict__ T, const double *__restrict__ Dinv,
                                                     const double *__restrict__ b, double *y, int32_t *flags,
                                                     uint64_t *ticket, uint64_t ticket_base, int32_t epoch, int upper,
                                                     int32_t *fail) {
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
    gf64 *gy = (gf64 *)y;
    gi32 *gflag = (gi32 *)flags;
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
        if (threadIdx.x == 0) {
            int64_t spins = 0;
            while (__hip_atomic_load(gflag + J, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1ll << 26)) {  // never expected: report instead of hanging the queue
                    atomicOr(fail, 2);
                    break;
                }
            }
        }
        __syncthreads();
        if (threadIdx.x < BT) {
            const int64_t gj = J * BT + threadIdx.x;
            ys[threadIdx.x] = gj < n ? __hip_atomic_load(gy + gj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
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
    if (part == 0 && gi < n) __hip_atomic_store(gy + gi, z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(gflag + I, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

void launch_band_sweep(int64_t n, int64_t nb, int64_t bl, int64_t bu, const double *T, const double *Dinv,
                       const double *b, double *y, int32_t *flags, uint64_t *ticket, uint64_t ticket_base,
                       int32_t epoch, int upper, int32_t *fail, hipStream_t st) {
    if (nb > 0)
        k_band_sweep<<<(unsigned)nb, BTPB, 0, st>>>(n, nb, bl, bu, T, Dinv, b, y, flags, ticket, ticket_base, epoch,
                                                   upper, fail);
}

}  // namespace pls
