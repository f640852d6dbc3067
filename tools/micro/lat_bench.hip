// Micro-benchmark: load latency and per-wave streaming throughput on MI355X
// (diagnostics for the latency-bound block sweeps).
//   chase:  one lane, dependent pointer chase over a buffer (HBM latency)
//   stream: one wave per block, K loads (4 B/lane) per step, D steps in flight
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__global__ void k_chase(const int64_t *next, int64_t start, int steps, int64_t *out, int64_t *tim) {
    int64_t p = start;
    const int64_t t0 = wall_clock64();
    for (int s = 0; s < steps; ++s) p = __builtin_nontemporal_load(next + p);
    const int64_t t1 = wall_clock64();
    out[0] = p;
    tim[0] = t1 - t0;
}

template <int K, bool NT>
__global__ void k_stream(const int *buf, int64_t n, int steps, int64_t *out, int64_t *tim) {
    const int lane = threadIdx.x & 63;
    int64_t off = (int64_t)blockIdx.x * 1048576;
    int a[4][K];
    int acc = 0;
    const int64_t t0 = wall_clock64();
    auto issue = [&](int s, int (&r)[K]) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t pos = (off + ((int64_t)s * K + k) * 64 + lane) & (n - 1);
            r[k] = NT ? __builtin_nontemporal_load(buf + pos) : buf[pos];
        }
    };
    issue(0, a[0]); issue(1, a[1]); issue(2, a[2]);
    for (int s = 0; s < steps; s += 4) {
        issue(s + 3, a[3]);
#pragma unroll
        for (int k = 0; k < K; ++k) acc += a[0][k];
        issue(s + 4, a[0]);
#pragma unroll
        for (int k = 0; k < K; ++k) acc += a[1][k];
        issue(s + 5, a[1]);
#pragma unroll
        for (int k = 0; k < K; ++k) acc += a[2][k];
        issue(s + 6, a[2]);
#pragma unroll
        for (int k = 0; k < K; ++k) acc += a[3][k];
    }
    const int64_t t1 = wall_clock64();
    if (acc == 123456789) out[lane] = acc;
    if (lane == 0) tim[blockIdx.x] = t1 - t0;
}

int main() {
    const int64_t n = (int64_t)1 << 28;  // 1 GiB of int32 / 2 GiB of int64 chase
    int64_t *next, *out, *tim;
    int *buf;
    hipMalloc(&next, n * sizeof(int64_t));
    hipMalloc(&buf, n * sizeof(int));
    hipMalloc(&out, 1024 * sizeof(int64_t));
    hipMalloc(&tim, 1024 * sizeof(int64_t));
    hipMemset(buf, 0, n * sizeof(int));
    // chase: stride of 1 MiB + 64 B through the buffer
    {
        int64_t *h = (int64_t *)malloc(n * sizeof(int64_t));
        const int64_t stride = 131072 + 8;
        for (int64_t i = 0; i < n; ++i) h[i] = (i + stride) % n;
        hipMemcpy(next, h, n * sizeof(int64_t), hipMemcpyHostToDevice);
        free(h);
    }
    int64_t ht[1024];
    for (int rep = 0; rep < 2; ++rep) {
        k_chase<<<1, 1>>>(next, 0, 2000, out, tim);
        hipDeviceSynchronize();
    }
    hipMemcpy(ht, tim, 8, hipMemcpyDeviceToHost);
    printf("chase (nt, 1 MiB stride): %.0f ns per dependent load\n", ht[0] * 10.0 / 2000);
    const int steps = 4000;
    auto run = [&](auto kern, const char *name, int K, int nb) {
        for (int rep = 0; rep < 2; ++rep) {
            kern<<<nb, 64>>>(buf, n, steps, out, tim);
            hipDeviceSynchronize();
        }
        hipMemcpy(ht, tim, nb * 8, hipMemcpyDeviceToHost);
        int64_t mx = 0;
        for (int b = 0; b < nb; ++b) mx = ht[b] > mx ? ht[b] : mx;
        const double us = mx * 0.01, per = us / steps;
        const double gbs = (double)nb * steps * K * 256 / (us * 1e-6) / 1e9;
        printf("%-10s K=%2d blocks %3d: %.3f us per step, %.1f GB/s per wave, %.1f GB/s total\n", name, K, nb, per,
               gbs / nb, gbs);
    };
    for (int nb : {1, 10, 256}) {
        run(k_stream<1, true>, "stream nt", 1, nb);
        run(k_stream<4, true>, "stream nt", 4, nb);
        run(k_stream<16, true>, "stream nt", 16, nb);
        run(k_stream<16, false>, "stream", 16, nb);
    }
    printf("err %s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
