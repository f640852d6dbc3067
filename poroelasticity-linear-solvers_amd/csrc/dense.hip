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

void launch_dense_invert(int64_t ld, double *M, double *D, int32_t *fail, hipStream_t st) {
    const int64_t nb = ld / DB;
    for (int64_t k = 0; k < nb; ++k) {
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
__global__ __launch_bounds__(256) void k_dense_gemv(int64_t n, int64_t ld, const double *__restrict__ M,
                                                    const double *__restrict__ x, double *__restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const int lane = threadIdx.x & 63;
    const double *row = M + i * ld;
    double acc = 0.0;
    const int64_t n2 = n & ~(int64_t)1;
    for (int64_t c = 2 * lane; c < n2; c += 128) {
        const dn_d2 m = __builtin_nontemporal_load(reinterpret_cast<const dn_d2 *>(row + c));
        acc += m.x * x[c];
        acc += m.y * x[c + 1];
    }
    if ((n & 1) && lane == 0) acc += row[n - 1] * x[n - 1];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) y[i] = acc;
}
void launch_dense_gemv(int64_t n, int64_t ld, const double *M, const double *x, double *y, hipStream_t st) {
    if (n > 0) k_dense_gemv<<<(unsigned)((n + 3) / 4), 256, 0, st>>>(n, ld, M, x, y);
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

}  // namespace pls
