// amg_host.hpp -- host-side sparse algebra shared by the AMG setups
// (amg.cpp: smoothed aggregation; boomeramg.cpp: classical AMG).
#pragma once
#include <algorithm>
#include <cstdint>
#include <atomic>
#include <thread>
#include <vector>

#include "runtime.hpp"

namespace pls {
namespace amgh {

// Host threads for the setup algebra (rows are independent, so results do
// not depend on the count): OMP_NUM_THREADS if set, else the hardware's, <= 64.
int setup_threads();

// fn(t, i0, i1) on T contiguous row ranges, one thread each
template <class F>
void parallel_rows(int64_t n, int T, F fn) {
    T = (int)std::max<int64_t>(1, std::min<int64_t>(T, n / 8));  // rows may be long (R = P^T)
    if (T == 1) {
        fn(0, (int64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(fn, t, n * t / T, n * (t + 1) / T);
    for (auto &x : th) x.join();
}

// fn(t, i0, i1) over blocks of `block` rows handed out to T threads on demand
// (rows of very different cost, results written per row); init(t) once per thread
template <class I, class F>
void parallel_dynamic(int64_t n, int T, int64_t block, I init, F fn) {
    T = (int)std::max<int64_t>(1, std::min<int64_t>(T, (n + block - 1) / block));
    std::atomic<int64_t> next{0};
    auto run = [&](int t) {
        init(t);
        for (int64_t i0; (i0 = next.fetch_add(block)) < n;) fn(t, i0, std::min(n, i0 + block));
    };
    if (T == 1) {
        run(0);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(run, t);
    for (auto &x : th) x.join();
}

HostCSR transpose(const HostCSR &A);
// Concatenate per-thread row ranges (ci/v/row lengths) into one CSR.
void concat_rows(HostCSR &C, std::vector<HostCSR> &part);
// C = A B in scipy's csr_matmat order (exact zero sums dropped, columns sorted)
HostCSR spgemm(const HostCSR &A, const HostCSR &B);
// Ac = P^T (A P), bitwise spgemm(R, spgemm(A, P)); false when nc^2 doubles exceed max_bytes
bool galerkin_fused(const HostCSR &A, const HostCSR &P, int64_t nc, double max_bytes, HostCSR &C);
// dense inverse by Gauss-Jordan with partial pivoting (coarsest level)
HostCSR dense_inverse(const HostCSR &A);
// SpMV layout for an AMG operator (SELL-64 for short rows, CSR otherwise)
void amg_layout(DevCSR &M, Ctx &c);

}  // namespace amgh
}  // namespace pls
