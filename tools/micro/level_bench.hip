// Micro-benchmark: per-level cost of the block-Jacobi LDS sweep's skeleton on
// one workgroup of 1024 threads (diagnostics for kernels.hip sweep2).
//   mode 0: __syncthreads() only
//   mode 1: + 2 waves do 7 dependent-address LDS reads and one LDS write
//   mode 2: + every wave issues 16 global loads per level, consumed 2 levels later
//   mode 3: mode 2 with only waves 0-1 loading
//   mode 4: mode 3 without the barrier
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(1024) void k_level(int mode, int levels, const int *col, const double *val,
                                                int64_t stride, double *out, int64_t *tim) {
    extern __shared__ double ys[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int t = threadIdx.x; t < 16384; t += 1024) ys[t] = 1.0 + t;
    __syncthreads();
    int c0[8], c1[8], c2[8];
    double v0[8], v1[8], v2[8];
    const int64_t wbase = (int64_t)blockIdx.x * levels * 16 * 64 * 8 + wave * 64 * 8;
    auto issue = [&](int g, int (&c)[8], double (&v)[8]) {
        const bool ld = mode == 2 || (mode >= 3 && wave < 2);
        const int64_t base = ld ? (wbase + (int64_t)g * 16 * 64 * 8) & (stride - 1) : 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            c[u] = __builtin_nontemporal_load(col + base + u * 64 + lane);
            v[u] = __builtin_nontemporal_load(val + base + u * 64 + lane);
        }
    };
    double acc = 0.0;
    auto level = [&](int g, const int (&c)[8], const double (&v)[8], int (&cn)[8], double (&vn)[8]) {
        if (mode >= 2) issue(g + 2, cn, vn);
        if (mode >= 1 && wave < 2) {
            double a = 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u) a += v[u] * ys[(c[u] + g * 64 + lane) & 16383];
            ys[(wave * 64 + lane + g * 128) & 16383] = a;
            acc += a;
        }
        if (mode != 4) __syncthreads();
    };
    int64_t t0 = wall_clock64();
    if (mode >= 2) { issue(0, c0, v0); issue(1, c1, v1); }
    else {
        for (int u = 0; u < 8; ++u) { c0[u] = c1[u] = c2[u] = u; v0[u] = v1[u] = v2[u] = 1.0; }
    }
    for (int g = 0; g < levels;) {
        level(g, c0, v0, c2, v2); if (++g >= levels) break;
        level(g, c1, v1, c0, v0); if (++g >= levels) break;
        level(g, c2, v2, c1, v1); if (++g >= levels) break;
    }
    int64_t t1 = wall_clock64();
    if (threadIdx.x == 0) tim[blockIdx.x] = t1 - t0;
    if (acc == 12345.0) out[threadIdx.x] = acc;
}

int main() {
    const int levels = 263;
    const int64_t stride = (int64_t)1 << 26;  // 64M entries
    int *col; double *val, *out; int64_t *tim;
    hipMalloc(&col, stride * sizeof(int) + 4096 * 64);
    hipMalloc(&val, stride * sizeof(double) + 8192 * 64);
    hipMemset(col, 0, stride * sizeof(int) + 4096 * 64);
    hipMemset(val, 0, stride * sizeof(double) + 8192 * 64);
    hipMalloc(&out, 1024 * sizeof(double));
    hipMalloc(&tim, 512 * sizeof(int64_t));
    hipFuncSetAttribute((const void *)k_level, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    for (int nb : {10, 256}) {
        for (int mode = 0; mode < 5; ++mode) {
            for (int rep = 0; rep < 2; ++rep) {
                k_level<<<nb, 1024, 131072>>>(mode, levels, col, val, stride, out, tim);
                hipDeviceSynchronize();
            }
            int64_t h[512];
            hipMemcpy(h, tim, nb * sizeof(int64_t), hipMemcpyDeviceToHost);
            int64_t mx = 0; for (int b = 0; b < nb; ++b) mx = h[b] > mx ? h[b] : mx;
            printf("blocks %3d mode %d: %.3f us per level (max over blocks)\n", nb, mode, mx * 0.01 / levels);
        }
    }
    printf("err %s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
