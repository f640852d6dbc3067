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

// Near-tile products for the sweeps: Gl[I] = Dl_I L_{I,I-1} (I >= 1) and
// Gu[I] = Du_I U_{I,I+1} (I <= nb - 2); blockIdx.y selects the triangle.
__global__ __launch_bounds__(BTPB) void k_band_near(int64_t nb, int64_t bl, int64_t bu, const double *T,
                                                    const double *Dl, const double *Du, double *Gl, double *Gu) {
    __shared__ double at[BT][BT + 1];
    __shared__ double b[BT][BT + 1];
    const int64_t I = blockIdx.x, W = bl + bu + 1;
    const bool up = blockIdx.y == 1;
    if (up ? (I >= nb - 1 || bu == 0) : (I < 1 || bl == 0)) return;
    const int64_t J = up ? I + 1 : I - 1;
    double acc[4][4];
    band_tile_mm((up ? Du : Dl) + I * TILE, T + (I * W + (J - I + bl)) * TILE, at, b, acc);
    double *C = (up ? Gu : Gl) + I * TILE;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) C[(ty + 16 * r) * BT + tx + 16 * q] = acc[r][q];
}

void launch_band_factor(int64_t nb, int64_t bl, int64_t bu, double *T, double *Dl, double *Du, double *Gl,
                        double *Gu, int32_t *fail, hipStream_t st) {
    if (nb <= 0) return;
    const int64_t W = bl + bu + 1;
    for (int64_t K = 0; K < nb; ++K) {
        k_band_diag<<<1, BTPB, 0, st>>>(W, bl, K, T, Dl, Du, fail);
        const int64_t rest = nb - 1 - K;
        const int64_t pl = bl < rest ? bl : rest, pu = bu < rest ? bu : rest;
        if (pl + pu == 0) continue;
        k_band_panels<<<(unsigned)(bl + pu), BTPB, 0, st>>>(nb, W, bl, K, T, Dl, Du);
        if (pl > 0 && pu > 0) k_band_update<<<dim3((unsigned)pu, (unsigned)pl), BTPB, 0, st>>>(nb, W, bl, K, T);
    }
    (void)hipMemsetAsync(Gl, 0, sizeof(double) * (size_t)(nb * TILE), st);
    (void)hipMemsetAsync(Gu, 0, sizeof(double) * (size_t)(nb * TILE), st);
    if (nb > 1) k_band_near<<<dim3((unsigned)nb, 2), BTPB, 0, st>>>(nb, bl, bu, T, Dl, Du, Gl, Gu);
}

// ------------------------------------------------------------------ sweeps --
typedef double bd_d2 __attribute__((ext_vector_type(2)));

// One triangle (upper = 0: forward with L, Dl, Gl; 1: backward with U, Du,
// Gu), walked in "positions" p (p = I forward, nb - 1 - I backward) so both
// directions read alike.  A workgroup of SR x 256 threads takes SR = 2
// consecutive positions (a super-row: one cross-workgroup hop per 128 rows);
// group g (4 waves) owns position p0 + g, its thread t owns row t / 4 and
// columns 16 (t % 4) .. +16 of every tile.  With bw tiles of the band on the
// solved side,
//     y_I = c_I - G_I y_near,   c_I = Dinv_I (b_I - sum_{J far} T_IJ y_J),
// so the chain from the neighbouring tile row's y to y_I is one preloaded
// tile product (G = Gl or Gu).  b and y have n entries (padding rows are 0
// and never stored); b != y.
// Hand-off (Guideline 16 R2, the data is the flag): y_I is published as 128
// 8-byte granules {epoch, 32 bits of y} in Gr (tile row I: Gr[128 I + 2 r +
// h], h = 0 low / 1 high half of row r), each written by ONE sc1 store; wave
// 0 re-reads a tile row's 128 granules with sc1 loads until every tag equals
// this sweep's epoch (bounded spin), then stages y_J in LDS.  The caller
// passes a fresh epoch (never 0; Gr starts zeroed) and the tickets drawn by
// earlier sweeps (band_sweep_tickets(nb) each) as ticket_base.
static constexpr int SR = 2;

__device__ __forceinline__ void band_stage(const gu64 *gr, int64_t J, uint32_t epoch, double *ys, int32_t *fail) {
    if (threadIdx.x < 64) {  // wave 0 sweeps tile row J's granules
        const int l = threadIdx.x;
        const gu64 *g = gr + J * 128 + 2 * l;
        uint64_t lo = 0, hi = 0;
        for (int64_t spins = 0;; ++spins) {
            lo = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            hi = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool ok = (uint32_t)(lo >> 32) == epoch && (uint32_t)(hi >> 32) == epoch;
            if (__all(ok)) break;
            if (spins > (1ll << 26)) {  // never expected: report instead of hanging the queue, and
                if (l == 0) atomicOr(fail, 2);  // poison y so the Krylov loop stops (DIVERGED_NANORINF)
                hi = 0x7ff80000ull;  // high half of a quiet NaN
                lo = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        ys[l] = __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
    }
    __syncthreads();
}

// partial row sum of a tile slice (16 entries per thread) against x in LDS
__device__ __forceinline__ double band_dot16(const bd_d2 (&m)[8], const double *x, int part) {
    double a = 0.0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        a += m[u].x * x[part * 16 + 2 * u];
        a += m[u].y * x[part * 16 + 2 * u + 1];
    }
    return a;
}
__device__ __forceinline__ double band_rowsum(double a) {  // over the 4 threads of a row; all get the sum
    a += __shfl_xor(a, 1);
    a += __shfl_xor(a, 2);
    return a;
}
__device__ __forceinline__ void band_load16(bd_d2 (&m)[8], const double *p, bool nt) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
        m[u] = nt ? __builtin_nontemporal_load(reinterpret_cast<const bd_d2 *>(p) + u)
                  : reinterpret_cast<const bd_d2 *>(p)[u];
}
// y_I to the granules and y (part-0 threads)
__device__ __forceinline__ void band_publish(gu64 *gr, int64_t I, int row, int64_t gi, int64_t n, double v,
                                             uint32_t epoch, double *y) {
    const uint64_t bits = gi < n ? (uint64_t)__double_as_longlong(v) : 0ull;  // padding rows publish 0
    const uint64_t tag = (uint64_t)epoch << 32;
    __hip_atomic_store(gr + I * 128 + 2 * row, tag | (bits & 0xffffffffull), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(gr + I * 128 + 2 * row + 1, tag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (gi < n) y[gi] = v;
}

__global__ __launch_bounds__(SR * 256) void k_band_sweep(int64_t n, int64_t nb, int64_t bl, int64_t bu,
                                                        const double *__restrict__ T, const double *__restrict__ Dinv,
                                                        const double *__restrict__ Gn, const double *__restrict__ b,
                                                        double *__restrict__ y, uint64_t *Gr, uint64_t *ticket,
                                                        uint64_t ticket_base, uint32_t epoch, int upper,
                                                        int32_t *fail, int64_t plen) {
    static_assert(SR == 2, "the chain below is written for two positions per workgroup");
    __shared__ int64_t sp;
    __shared__ double ys[BT];
    __shared__ double rs[SR][BT];
    __shared__ double y0[BT];
    if (threadIdx.x == 0) sp = (int64_t)(atomicAdd((unsigned long long *)ticket, 1ull) - ticket_base);
    __syncthreads();
    const int64_t nsr = (nb + SR - 1) / SR;
    if (sp < 0 || sp >= nsr) return;  // uniform
    const int64_t p0 = sp * SR;
    // SPIKE partitions (plen > 0, a multiple of SR): the chain restarts at the
    // first position of every partition (couplings to the previous partition
    // are applied afterwards through the spikes)
    const int64_t ps = plen > 0 ? (p0 / plen) * plen : 0;
    const int g = threadIdx.x >> 8, lt = threadIdx.x & 255, row = lt >> 2, part = lt & 3;
    const int64_t W = bl + bu + 1, bw = upper ? bu : bl;  // tiles on the solved side
    const int64_t pI = p0 + g;
    const bool act = pI < nb;
    const int64_t I = upper ? nb - 1 - pI : pI;
    const int64_t gi = I * BT + row;
    gu64 *gr = (gu64 *)Gr;
    auto tile_row = [&](int64_t pJ) { return upper ? nb - 1 - pJ : pJ; };
    auto tile = [&](int64_t pJ) { return T + (I * W + (tile_row(pJ) - I + bl)) * TILE + row * BT + part * 16; };
    // off the chain: b, Dinv and the near-tile product
    const bool has_near = act && bw >= 1 && pI >= 1 && pI - 1 >= ps;
    double bi = 0.0;
    bd_d2 dm[8], gm[8];
    if (act) {
        bi = gi < n ? b[gi] : 0.0;
        band_load16(dm, Dinv + I * TILE + row * BT + part * 16, false);
    }
    if (has_near) band_load16(gm, Gn + I * TILE + row * BT + part * 16, false);
    // far tiles preceding the super-row: positions [p0 - bw, p0 - 2]; group g
    // uses [pI - bw, pI - 2]
    double acc = 0.0;
    for (int64_t pJ = (p0 - bw > ps ? p0 - bw : ps); pJ <= p0 - 2; ++pJ) {
        const bool use = act && pJ >= pI - bw;
        bd_d2 m[8];
        if (use) band_load16(m, tile(pJ), true);
        band_stage(gr, tile_row(pJ), epoch, ys, fail);
        if (use) acc += band_dot16(m, ys, part);
        __syncthreads();  // ys is refilled next
    }
    // group 0: c_0 = Dinv (b - far); group 1 loads its tile at p0 - 1 (far
    // for it, near for group 0)
    if (g == 0 && act) {
        const double r = band_rowsum(acc);
        if (part == 0) rs[0][row] = bi - r;
    }
    bd_d2 m1[8];
    const bool use1 = act && g == 1 && p0 > ps && p0 - 1 >= pI - bw;
    if (use1) band_load16(m1, tile(p0 - 1), true);
    __syncthreads();
    double c0 = 0.0;
    if (g == 0 && act) c0 = band_rowsum(band_dot16(dm, rs[0], part));
    if (p0 > ps && bw >= 1) {
        band_stage(gr, tile_row(p0 - 1), epoch, ys, fail);  // the cross-workgroup hop
        if (g == 0 && act) {
            const double v = c0 - band_rowsum(band_dot16(gm, ys, part));
            if (part == 0) {
                y0[row] = v;
                band_publish(gr, I, row, gi, n, v, epoch, y);
            }
        }
        if (use1) acc += band_dot16(m1, ys, part);
    } else if (g == 0 && act && part == 0) {  // nothing near precedes position p0
        y0[row] = c0;
        band_publish(gr, I, row, gi, n, c0, epoch, y);
    }
    // group 1: c_1, then its near tile against group 0's y (through LDS)
    if (g == 1 && act) {
        const double r = band_rowsum(acc);
        if (part == 0) rs[1][row] = bi - r;
    }
    __syncthreads();
    if (g == 1 && act) {
        const double c1 = band_rowsum(band_dot16(dm, rs[1], part));
        const double v = has_near ? c1 - band_rowsum(band_dot16(gm, y0, part)) : c1;
        if (part == 0) band_publish(gr, I, row, gi, n, v, epoch, y);
    }
}

int64_t band_sweep_tickets(int64_t nb) { return (nb + SR - 1) / SR; }

void launch_band_sweep(int64_t n, int64_t nb, int64_t bl, int64_t bu, const double *T, const double *Dinv,
                       const double *Gn, const double *b, double *y, uint64_t *Gr, uint64_t *ticket,
                       uint64_t ticket_base, uint32_t epoch, int upper, int32_t *fail, hipStream_t st, int64_t plen) {
    if (nb > 0)
        k_band_sweep<<<(unsigned)band_sweep_tickets(nb), SR * 256, 0, st>>>(n, nb, bl, bu, T, Dinv, Gn, b, y, Gr,
                                                                            ticket, ticket_base, epoch, upper, fail,
                                                                            plen);
}

// ------------------------------------------------------------------ SPIKE --
// Partitioned triangle solve.  Positions (as in the sweep) are cut into
// partitions of plen positions (plen >= bw, a multiple of SR).  With t_k the
// solution on the last bw positions of partition k - 1 (its "tail"), the
// solution on partition k is  y = z - W t_k,  where z is the partition's own
// chain (k_band_sweep with plen: couplings to earlier partitions dropped) and
// the spikes  W[p][c] = Dinv_p (T(p, q_c) - sum_{p' in k, p - bw <= p' < p}
// T(p, p') W[p'][c])  (q_c = first position of k - bw + c; T(p, q_c) = 0
// outside the band) are formed once at setup, one tile GEMM chain per
// (partition, c) in parallel.  Per sweep: the partitions' chains run
// concurrently (plen / SR hops instead of nb / SR), then the tails are
// corrected partition by partition (P - 2 small launches), then every other
// position in one bandwidth-bound pass.  W takes nb x bw tiles.
__device__ __forceinline__ void band_tile_mac(const double *A, const double *B, double (*at)[BT + 1],
                                              double (*b)[BT + 1], double acc[4][4]) {
    __syncthreads();  // the previous product is done with the staging tiles
    for (int t = threadIdx.x; t < BT * BT; t += BTPB) {
        const int r = t / BT, cc = t % BT;
        at[cc][r] = A[t];
        b[r][cc] = B[t];
    }
    __syncthreads();
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
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

// spikes of position offset t in every partition k >= 1: blockIdx.x = c, blockIdx.y = k - 1
__global__ __launch_bounds__(BTPB) void k_spike_w(int64_t nb, int64_t bl, int64_t bu, int upper, int64_t plen,
                                                  int64_t t, const double *__restrict__ T,
                                                  const double *__restrict__ Dinv, double *__restrict__ Wt) {
    __shared__ double at[BT][BT + 1];
    __shared__ double bb[BT][BT + 1];
    __shared__ double cs[BT][BT + 1];
    const int64_t W = bl + bu + 1, bw = upper ? bu : bl;
    const int64_t c = blockIdx.x, k = (int64_t)blockIdx.y + 1, k0 = k * plen;
    const int64_t pI = k0 + t, kend = (k0 + plen < nb) ? k0 + plen : nb;
    if (pI >= kend) return;
    auto trow = [&](int64_t p) { return upper ? nb - 1 - p : p; };
    auto tile = [&](int64_t pa, int64_t pb) { return T + (trow(pa) * W + (trow(pb) - trow(pa) + bl)) * TILE; };
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    double acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[r][q] = 0.0;
    // sum_{p'} T(pI, p') W[p'][c], p' ascending
    for (int64_t pJ = (pI - bw > k0 ? pI - bw : k0); pJ < pI; ++pJ)
        band_tile_mac(tile(pI, pJ), Wt + (pJ * bw + c) * TILE, at, bb, acc);
    // cs = T(pI, q_c) - sum
    const int64_t qc = k0 - bw + c;
    const bool in_band = qc >= 0 && qc >= pI - bw;
    const double *Tq = in_band ? tile(pI, qc) : nullptr;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = ty + 16 * r, j = tx + 16 * q;
            cs[i][j] = (in_band ? Tq[i * BT + j] : 0.0) - acc[r][q];
        }
    __syncthreads();
    // W[pI][c] = Dinv(pI) cs
    const double *D = Dinv + trow(pI) * TILE;
    double o[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) o[r][q] = 0.0;
    for (int kk = 0; kk < BT; ++kk) {
        double dv[4], cv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) dv[r] = D[(ty + 16 * r) * BT + kk];
#pragma unroll
        for (int q = 0; q < 4; ++q) cv[q] = cs[kk][tx + 16 * q];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) o[r][q] += dv[r] * cv[q];
    }
    double *out = Wt + (pI * bw + c) * TILE;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) out[(ty + 16 * r) * BT + tx + 16 * q] = o[r][q];
}

void launch_spike_setup(int64_t nb, int64_t bl, int64_t bu, int upper, int64_t plen, const double *T,
                        const double *Dinv, double *Wt, hipStream_t st) {
    const int64_t bw = upper ? bu : bl, P = (nb + plen - 1) / plen;
    if (P < 2 || bw == 0) return;
    for (int64_t t = 0; t < plen; ++t)
        k_spike_w<<<dim3((unsigned)bw, (unsigned)(P - 1)), BTPB, 0, st>>>(nb, bl, bu, upper, plen, t, T, Dinv, Wt);
}

// y_p -= sum_c W[p][c] y_{q_c} for the positions p0 + blockIdx.x (one workgroup
// each; thread t: row t / 4, columns 16 (t % 4) .. +16 of every tile; sums in
// c, then column order, then the 4 parts).  mode 0: the tail positions of
// partition k (p0 = its last bw positions); mode 1: every position of every
// partition k >= 1 except the tails already corrected (p0 = 0, all nb).
__global__ __launch_bounds__(BTPB) void k_spike_correct(int64_t n, int64_t nb, int64_t bw, int upper, int64_t plen,
                                                        int64_t p0, int mode, const double *__restrict__ Wt,
                                                        double *__restrict__ y) {
    __shared__ double ts[BT];
    const int64_t pI = p0 + blockIdx.x;
    if (pI >= nb) return;
    const int64_t k = pI / plen, k0 = k * plen, kend = (k0 + plen < nb) ? k0 + plen : nb;
    const int64_t P = (nb + plen - 1) / plen;
    if (k == 0) return;
    if (mode == 1 && k < P - 1 && pI >= kend - bw) return;  // a tail: done by mode 0
    auto trow = [&](int64_t p) { return upper ? nb - 1 - p : p; };
    const int lt = threadIdx.x, row = lt >> 2, part = lt & 3;
    double s = 0.0;
    for (int64_t c = 0; c < bw; ++c) {
        const int64_t qc = k0 - bw + c;
        __syncthreads();
        if (lt < BT) {
            const int64_t gq = trow(qc) * BT + lt;
            ts[lt] = (qc >= 0 && gq < n) ? y[gq] : 0.0;
        }
        __syncthreads();
        const bd_d2 *w = reinterpret_cast<const bd_d2 *>(Wt + (pI * bw + c) * TILE + row * BT + part * 16);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const bd_d2 m = __builtin_nontemporal_load(w + u);
            s += m.x * ts[part * 16 + 2 * u];
            s += m.y * ts[part * 16 + 2 * u + 1];
        }
    }
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    const int64_t gi = trow(pI) * BT + row;
    if (part == 0 && gi < n) y[gi] = y[gi] - s;
}

// The tails are on the sequential path: their bw x bw tiles per position are
// spread over SPIKE_G workgroups (SPIKE_CG spike tiles each) whose partial
// row sums a second launch adds in group order.
static constexpr int SPIKE_CG = 4;
__global__ __launch_bounds__(BTPB) void k_spike_tail_part(int64_t n, int64_t nb, int64_t bw, int upper, int64_t plen,
                                                          int64_t p0, const double *__restrict__ Wt,
                                                          const double *__restrict__ y, double *__restrict__ part_out) {
    __shared__ double ts[BT];
    const int64_t pI = p0 + blockIdx.x, k0 = (pI / plen) * plen;
    const int64_t c0 = (int64_t)blockIdx.y * SPIKE_CG, c1 = (c0 + SPIKE_CG < bw) ? c0 + SPIKE_CG : bw;
    auto trow = [&](int64_t p) { return upper ? nb - 1 - p : p; };
    const int lt = threadIdx.x, row = lt >> 2, part = lt & 3;
    double s = 0.0;
    for (int64_t c = c0; c < c1; ++c) {
        const int64_t qc = k0 - bw + c;
        __syncthreads();
        if (lt < BT) {
            const int64_t gq = trow(qc) * BT + lt;
            ts[lt] = (qc >= 0 && gq < n) ? y[gq] : 0.0;
        }
        __syncthreads();
        const bd_d2 *w = reinterpret_cast<const bd_d2 *>(Wt + (pI * bw + c) * TILE + row * BT + part * 16);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const bd_d2 m = __builtin_nontemporal_load(w + u);
            s += m.x * ts[part * 16 + 2 * u];
            s += m.y * ts[part * 16 + 2 * u + 1];
        }
    }
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    if (part == 0) part_out[((int64_t)blockIdx.x * gridDim.y + blockIdx.y) * BT + row] = s;
}
__global__ __launch_bounds__(BT) void k_spike_tail_fin(int64_t n, int64_t nb, int upper, int64_t p0, int G,
                                                       const double *__restrict__ part_in, double *__restrict__ y) {
    const int64_t pI = p0 + blockIdx.x;
    const int row = threadIdx.x;
    double s = 0.0;
    for (int g = 0; g < G; ++g) s += part_in[((int64_t)blockIdx.x * G + g) * BT + row];
    const int64_t gi = (upper ? nb - 1 - pI : pI) * BT + row;
    if (gi < n) y[gi] = y[gi] - s;
}

int64_t spike_scratch_doubles(int64_t bw) { return bw * ((bw + SPIKE_CG - 1) / SPIKE_CG) * BT; }

void launch_spike_apply(int64_t n, int64_t nb, int64_t bw, int upper, int64_t plen, const double *Wt, double *y,
                        double *scratch, hipStream_t st) {
    const int64_t P = (nb + plen - 1) / plen;
    if (P < 2 || bw == 0) return;
    const int G = (int)((bw + SPIKE_CG - 1) / SPIKE_CG);
    for (int64_t k = 1; k + 1 < P; ++k) {  // tails, in partition order (each needs the previous one final)
        const int64_t p0 = (k + 1) * plen - bw;
        k_spike_tail_part<<<dim3((unsigned)bw, (unsigned)G), BTPB, 0, st>>>(n, nb, bw, upper, plen, p0, Wt, y,
                                                                            scratch);
        k_spike_tail_fin<<<(unsigned)bw, BT, 0, st>>>(n, nb, upper, p0, G, scratch, y);
    }
    k_spike_correct<<<(unsigned)nb, BTPB, 0, st>>>(n, nb, bw, upper, plen, 0, 1, Wt, y);
}

}  // namespace pls
