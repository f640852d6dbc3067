// amg.cpp -- smoothed-aggregation algebraic multigrid (PCGAMG-like), the
// device preconditioner behind -pc_type gamg and, by default, the stand-in for
// -pc_type hypre (BoomerAMG is absent from this image; reference drivers
// footing.py:73, swelling.py:70, swelling-3d.py:71 default "inner pc type" to
// hypre, and petsc-options-inexact selects it for the s_/f_/p_ blocks).
//
// The algorithm is specified in oracle/amg.py (the test oracle); the setup
// here reproduces it bit for bit -- every host sum runs in the order scipy's
// sparsetools use (row-storage order, left to right, no contraction) and the
// spectral estimate is rounded to float -- so the hierarchy (aggregates, P,
// coarse operators) is identical to the oracle's and only the device V-cycle
// rounding differs.
//
// Setup runs once on the host (aggregation is sequential by definition);
// every level's A, P, R = P^T is then device resident in the SpMV layout and
// one V-cycle is a fixed sequence of SpMVs and fused Chebyshev steps on the
// context's stream; the coarsest level is a dense inverse (one SpMV) up to
// 1024 rows, the device LU pipeline above that.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <thread>

#include "amg_host.hpp"

#pragma clang fp contract(off)

namespace pls {
namespace amgh {

HostCSR transpose(const HostCSR &A) {
    HostCSR T;
    T.nrows = A.ncols;
    T.ncols = A.nrows;
    const int64_t n = A.nrows, m = A.ncols, nnz = (int64_t)A.ci.size();
    T.rp.assign(m + 1, 0);
    T.ci.resize(nnz);
    T.v.resize(nnz);
    // per thread column counts over its row range, thread-major offsets inside every
    // column, then every thread fills its rows: each column's rows stay ascending
    int Tn = setup_threads();
    if (m > 0) Tn = (int)std::max<int64_t>(1, std::min<int64_t>(Tn, nnz / (2 * m)));
    if (nnz < (int64_t)1 << 20 || n < 1024) Tn = 1;
    std::vector<int64_t> r0(Tn + 1);
    for (int t = 0; t <= Tn; ++t) r0[t] = n * t / Tn;
    std::vector<std::vector<int64_t>> cnt(Tn);
    auto run = [&](auto fn) {
        std::vector<std::thread> th;
        for (int t = 0; t < Tn; ++t) th.emplace_back(fn, t);
        for (auto &x : th) x.join();
    };
    run([&](int t) {
        cnt[t].assign(m, 0);
        for (int64_t k = A.rp[r0[t]]; k < A.rp[r0[t + 1]]; ++k) ++cnt[t][A.ci[k]];
    });
    for (int64_t j = 0; j < m; ++j) {
        int64_t o = T.rp[j];
        for (int t = 0; t < Tn; ++t) {
            const int64_t c = cnt[t][j];
            cnt[t][j] = o;
            o += c;
        }
        T.rp[j + 1] = o;
    }
    run([&](int t) {
        std::vector<int64_t> &pos = cnt[t];
        for (int64_t i = r0[t]; i < r0[t + 1]; ++i)
            for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                const int64_t q = pos[A.ci[k]]++;
                T.ci[q] = (int32_t)i;
                T.v[q] = A.v[k];
            }
    });
    return T;  // rows ascending (i visited in order)
}

// Host threads for the setup algebra (rows are independent, so results do
// not depend on the count): OMP_NUM_THREADS if set, else the hardware's, <= 64.
int setup_threads() {
    int t = (int)std::thread::hardware_concurrency();
    if (const char *e = std::getenv("OMP_NUM_THREADS")) t = std::atoi(e);
    return std::max(1, std::min(t, 64));
}

// Concatenate per-thread row ranges (ci/v/row lengths) into one CSR (each
// part copied into place by a thread of its own).
void concat_rows(HostCSR &C, std::vector<HostCSR> &part) {
    const size_t T = part.size();
    std::vector<int64_t> row0(T + 1, 0), nz0(T + 1, 0);
    for (size_t t = 0; t < T; ++t) {
        row0[t + 1] = row0[t] + (part[t].rp.empty() ? 0 : (int64_t)part[t].rp.size() - 1);
        nz0[t + 1] = nz0[t] + (int64_t)part[t].ci.size();
    }
    C.rp.assign(row0[T] + 1, 0);
    C.ci.resize(nz0[T]);
    C.v.resize(nz0[T]);
    std::vector<std::thread> th;
    for (size_t t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            HostCSR &p = part[t];
            for (size_t k = 1; k < p.rp.size(); ++k) C.rp[row0[t] + k] = nz0[t] + p.rp[k];
            std::copy(p.ci.begin(), p.ci.end(), C.ci.begin() + nz0[t]);
            std::copy(p.v.begin(), p.v.end(), C.v.begin() + nz0[t]);
            HostCSR().rp.swap(p.rp);
            hvec<int32_t>().swap(p.ci);
            hvec<double>().swap(p.v);
        });
    for (auto &x : th) x.join();
}

// C = A B, row i accumulating over A's row in storage order (csr_matmat);
// exact zero sums dropped; columns sorted.  Rows in parallel.
void spgemm_rows(const HostCSR &A, const HostCSR &B, int64_t i0, int64_t i1, HostCSR &C) {
    C.rp.assign(1, 0);
    std::vector<double> acc(B.ncols, 0.0);
    std::vector<char> mark(B.ncols, 0);
    std::vector<int32_t> cols;
    for (int64_t i = i0; i < i1; ++i) {
        cols.clear();
        for (int64_t kk = A.rp[i]; kk < A.rp[i + 1]; ++kk) {
            const int32_t k = A.ci[kk];
            const double a = A.v[kk];
            for (int64_t jj = B.rp[k]; jj < B.rp[k + 1]; ++jj) {
                const int32_t j = B.ci[jj];
                if (!mark[j]) {
                    mark[j] = 1;
                    acc[j] = 0.0;
                    cols.push_back(j);
                }
                acc[j] += a * B.v[jj];
            }
        }
        std::sort(cols.begin(), cols.end());
        for (int32_t j : cols) {
            if (acc[j] != 0.0) {
                C.ci.push_back(j);
                C.v.push_back(acc[j]);
            }
            mark[j] = 0;
        }
        C.rp.push_back((int64_t)C.ci.size());
    }
}

HostCSR spgemm(const HostCSR &A, const HostCSR &B) {
    HostCSR C;
    C.nrows = A.nrows;
    C.ncols = B.ncols;
    const int T = setup_threads();
    std::vector<HostCSR> part(T);
    parallel_rows(A.nrows, T, [&](int t, int64_t i0, int64_t i1) { spgemm_rows(A, B, i0, i1, part[t]); });
    concat_rows(C, part);
    return C;
}

// Galerkin product Ac = R (A P) with R = P^T, bitwise equal to
// spgemm(R, spgemm(A, P)) (csr_matmat twice):
//  * (AP)_kb is summed exactly as there (A's row k in storage order, P's rows
//    in order), exact zeros dropped;
//  * every Ac entry (a, b) sums R_ak (AP)_kb over R's row a in storage order,
//    k ascending -- the same sequence as visiting fine rows k in order and
//    scattering P_ka (AP)_kb.
// This fused outer-product form never materialises AP (~950 entries per row
// at N=59: ~57 GB) nor sorts its rows, and streams A and P once per thread.
// Threads own coarse-row ranges with a dense accumulator each (a fine row
// whose P row touches a range is expanded by that range's thread), so it is
// used while nc^2 doubles stay small (max_bytes).
bool galerkin_fused(const HostCSR &A, const HostCSR &P, int64_t nc, double max_bytes, HostCSR &C) {
    if ((double)nc * (double)nc * 8.0 > max_bytes) return false;
    // the dense slabs (nc^2 doubles, zeroed and scanned) only pay when A P
    // would be big: a mildly coarsened level (nc ~ n / 3) goes row-wise
    if ((double)nc * (double)nc > 4.0 * (double)A.ci.size()) return false;
    C.nrows = C.ncols = nc;
    const int T = (int)std::max<int64_t>(1, std::min<int64_t>(setup_threads(), nc));
    std::vector<HostCSR> part(T);
    // coarse-row ranges: equal shares of the (AP)_k work (a fine row's |A_k|
    // spread over its P row's coarse points), each boundary then moved within
    // +-1/4 share to where the fewest fine rows straddle it (a straddling row's
    // (AP)_k is computed by both threads)
    std::vector<int64_t> bound(T + 1, 0);
    bound[T] = nc;
    if (T > 1) {
        std::vector<double> w(nc + 1, 0.0);
        std::vector<int64_t> cross(nc + 1, 0);
        for (int64_t k = 0; k < P.nrows; ++k) {
            const int64_t b = P.rp[k], e = P.rp[k + 1];
            if (e == b) continue;
            const double c = (double)(A.rp[k + 1] - A.rp[k]) / (double)(e - b);
            for (int64_t q = b; q < e; ++q) w[P.ci[q] + 1] += c;
            ++cross[P.ci[b] + 1];  // straddles boundaries a with P.ci[b] < a <= P.ci[e - 1]
            --cross[P.ci[e - 1] + 1];
        }
        for (int64_t a = 0; a < nc; ++a) {
            w[a + 1] += w[a];
            cross[a + 1] += cross[a];
        }
        int64_t a = 0;
        for (int t = 1; t < T; ++t) {
            const double target = w[nc] * t / T;
            while (a < nc && w[a] < target) ++a;
            const int64_t lo = std::max<int64_t>(bound[t - 1] + 1, a - nc / (4 * T)), hi = std::min<int64_t>(nc - 1, a + nc / (4 * T));
            int64_t best = std::max<int64_t>(bound[t - 1] + 1, std::min<int64_t>(a, nc - 1));
            for (int64_t x = lo; x <= hi; ++x)
                if (cross[x] < cross[best]) best = x;
            bound[t] = std::min<int64_t>(best, nc);
        }
        for (int t = 1; t <= T; ++t) bound[t] = std::max(bound[t], bound[t - 1]);
    }
    std::vector<int64_t> ncomp(T, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) {
        th.emplace_back([&, t] {
            const int64_t a0 = bound[t], a1 = bound[t + 1];
            hvec<double> acc((size_t)((a1 - a0) * nc), 0.0);  // (huge pages: the scatter's rows are 120 KB apart)
            std::vector<double> ap(nc, 0.0);
            std::vector<uint8_t> mark(nc, 0);
            std::vector<int32_t> cols(nc + 1);
            for (int64_t k = 0; k < P.nrows; ++k) {
                bool touch = false;
                for (int64_t q = P.rp[k]; q < P.rp[k + 1] && !touch; ++q) touch = P.ci[q] >= a0 && P.ci[q] < a1;
                if (!touch) continue;
                ++ncomp[t];
                // (AP)_k, as spgemm_rows sums it (ap is all zero between rows;
                // the touched list grows branch-free)
                int64_t ncol = 0;
                for (int64_t kk = A.rp[k]; kk < A.rp[k + 1]; ++kk) {
                    const int32_t kp = A.ci[kk];
                    const double av = A.v[kk];
                    for (int64_t jj = P.rp[kp]; jj < P.rp[kp + 1]; ++jj) {
                        const int32_t b = P.ci[jj];
                        cols[ncol] = b;
                        ncol += mark[b] ^ 1;
                        mark[b] = 1;
                        ap[b] += av * P.v[jj];
                    }
                }
                for (int64_t q = P.rp[k]; q < P.rp[k + 1]; ++q) {
                    const int64_t a = P.ci[q];
                    if (a < a0 || a >= a1) continue;
                    const double p = P.v[q];
                    double *row = acc.data() + (a - a0) * nc;
                    for (int64_t u = 0; u < ncol; ++u) {
                        const int32_t b = cols[u];
                        if (ap[b] != 0.0) row[b] += p * ap[b];
                    }
                }
                for (int64_t u = 0; u < ncol; ++u) {
                    mark[cols[u]] = 0;
                    ap[cols[u]] = 0.0;
                }
            }
            HostCSR &out = part[t];
            out.rp.assign(1, 0);
            for (int64_t a = a0; a < a1; ++a) {
                const double *row = acc.data() + (a - a0) * nc;
                for (int64_t b = 0; b < nc; ++b)
                    if (row[b] != 0.0) {
                        out.ci.push_back((int32_t)b);
                        out.v.push_back(row[b]);
                    }
                out.rp.push_back((int64_t)out.ci.size());
            }
        });
    }
    for (auto &x : th) x.join();
    if (std::getenv("PLS_AMG_TRACE")) {
        int64_t tot = 0;
        for (int64_t x : ncomp) tot += x;
        fprintf(stderr, "[galerkin_fused] %d threads: (AP)_k rows formed %lld for %lld fine rows\n", T, (long long)tot,
                (long long)P.nrows);
    }
    concat_rows(C, part);
    return true;
}

// oracle/amg.py aggregate(): symmetric strength graph W = |A| + |A|^T (off
// diagonal, zero weights dropped), three deterministic passes.
std::vector<int32_t> aggregate(const HostCSR &A, double theta, int32_t &na) {
    const int64_t n = A.nrows;
    std::vector<double> d(n, 0.0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k)
            if (A.ci[k] == i) d[i] = std::fabs(A.v[k]);
    const HostCSR T = transpose(A);
    std::vector<int64_t> wp(n + 1, 0);
    std::vector<int32_t> wj;
    std::vector<double> ww;
    wj.reserve(A.ci.size());
    ww.reserve(A.ci.size());
    for (int64_t i = 0; i < n; ++i) {
        int64_t a = A.rp[i], ae = A.rp[i + 1], t = T.rp[i], te = T.rp[i + 1];
        while (a < ae || t < te) {
            int32_t j;
            double w;
            if (t >= te || (a < ae && A.ci[a] < T.ci[t])) {
                j = A.ci[a];
                w = std::fabs(A.v[a]) + 0.0;
                ++a;
            } else if (a >= ae || T.ci[t] < A.ci[a]) {
                j = T.ci[t];
                w = 0.0 + std::fabs(T.v[t]);
                ++t;
            } else {
                j = A.ci[a];
                w = std::fabs(A.v[a]) + std::fabs(T.v[t]);
                ++a;
                ++t;
            }
            if (j == i || w == 0.0) continue;
            if (!(w > 2.0 * theta * std::sqrt(d[i] * d[j]))) continue;
            wj.push_back(j);
            ww.push_back(w);
        }
        wp[i + 1] = (int64_t)wj.size();
    }
    std::vector<int32_t> agg(n, -1);
    na = 0;
    for (int64_t i = 0; i < n; ++i) {  // pass 1
        if (agg[i] >= 0) continue;
        bool free_nb = true;
        for (int64_t k = wp[i]; k < wp[i + 1] && free_nb; ++k) free_nb = agg[wj[k]] < 0;
        if (!free_nb) continue;
        agg[i] = na;
        for (int64_t k = wp[i]; k < wp[i + 1]; ++k) agg[wj[k]] = na;
        ++na;
    }
    const std::vector<int32_t> agg1 = agg;
    for (int64_t i = 0; i < n; ++i) {  // pass 2
        if (agg1[i] >= 0) continue;
        int64_t best = -1;
        double bw = -1.0;
        for (int64_t k = wp[i]; k < wp[i + 1]; ++k)
            if (agg1[wj[k]] >= 0 && ww[k] > bw) {
                best = wj[k];
                bw = ww[k];
            }
        if (best >= 0) agg[i] = agg1[best];
    }
    for (int64_t i = 0; i < n; ++i)  // pass 3
        if (agg[i] < 0) agg[i] = na++;
    return agg;
}

std::vector<double> jacobi_dinv(const HostCSR &A) {
    std::vector<double> dinv(A.nrows, 1.0);
    for (int64_t i = 0; i < A.nrows; ++i)
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k)
            if (A.ci[k] == i && A.v[k] != 0.0) dinv[i] = 1.0 / A.v[k];
    return dinv;
}

// power iteration on D^-1 A (oracle power_lambda), rounded to float so that
// the hierarchy does not depend on the norms' summation order
double power_lambda(const HostCSR &A, const std::vector<double> &dinv, int steps) {
    const int64_t n = A.nrows;
    std::vector<double> v(n, 1.0), w(n);
    double lam = 1.0;
    const int T = setup_threads();
    for (int s = 0; s < steps; ++s) {
        parallel_rows(n, T, [&](int, int64_t i0, int64_t i1) {
            for (int64_t i = i0; i < i1; ++i) {
                double acc = 0.0;
                for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) acc += A.v[k] * v[A.ci[k]];
                w[i] = dinv[i] * acc;
            }
        });
        double nw = 0.0, nv = 0.0;
        for (int64_t i = 0; i < n; ++i) {
            nw += w[i] * w[i];
            nv += v[i] * v[i];
        }
        nw = std::sqrt(nw);
        nv = std::sqrt(nv);
        if (nw == 0.0) return 1.0;
        lam = nw / nv;
        for (int64_t i = 0; i < n; ++i) v[i] = w[i] / nw;
    }
    return (double)(float)lam;
}

// dense inverse by Gauss-Jordan with partial pivoting (coarsest level)
HostCSR dense_inverse(const HostCSR &A) {
    const int64_t n = A.nrows;
    std::vector<double> M(n * n, 0.0), X(n * n, 0.0);
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) M[i * n + A.ci[k]] = A.v[k];
        X[i * n + i] = 1.0;
    }
    for (int64_t c = 0; c < n; ++c) {
        int64_t p = c;
        for (int64_t r = c + 1; r < n; ++r)
            if (std::fabs(M[r * n + c]) > std::fabs(M[p * n + c])) p = r;
        if (M[p * n + c] == 0.0) throw Error("AMG: singular coarsest-level matrix");
        if (p != c)
            for (int64_t j = 0; j < n; ++j) {
                std::swap(M[p * n + j], M[c * n + j]);
                std::swap(X[p * n + j], X[c * n + j]);
            }
        const double inv = 1.0 / M[c * n + c];
        for (int64_t j = 0; j < n; ++j) {
            M[c * n + j] *= inv;
            X[c * n + j] *= inv;
        }
        for (int64_t r = 0; r < n; ++r) {
            if (r == c) continue;
            const double f = M[r * n + c];
            if (f == 0.0) continue;
            for (int64_t j = 0; j < n; ++j) {
                M[r * n + j] -= f * M[c * n + j];
                X[r * n + j] -= f * X[c * n + j];
            }
        }
    }
    HostCSR D;
    D.nrows = D.ncols = n;
    D.rp.resize(n + 1);
    D.ci.resize(n * n);
    D.v.assign(X.begin(), X.end());
    for (int64_t i = 0; i <= n; ++i) D.rp[i] = i * n;
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n; ++j) D.ci[i * n + j] = (int32_t)j;
    return D;
}

// SpMV layout for an AMG operator: SELL-64 for short rows; matrices of few
// long rows (R = P^T, Galerkin coarse operators, the dense coarsest inverse)
// stay CSR and take the workgroup-per-row kernel.
void amg_layout(DevCSR &M, Ctx &c) {
    M.rcm_auto = false;  // Galerkin operators: the RCM relabelling is for caller (FE) blocks
    // short rows (interpolation P: ~7 per row) stay CSR, 8 lanes per row: in
    // SELL-64 a slice's few entries per lane leave each wave one dependent
    // round trip per slice (P e at N=59: 0.34-0.44 ms for 37M entries)
    if (M.nrows > 0 && M.nnz < 128 * M.nrows && (double)M.nnz >= c.amg_csr_below * (double)M.nrows) build_sell(M, c);
}

}  // namespace amgh

namespace {
using namespace amgh;

struct AmgLevel {
    const DevCSR *A = nullptr;      // level 0: the PC's matrix; else Aown
    std::unique_ptr<DevCSR> Aown;
    DevCSR P, R;
    DBuf<double> dinv;
    int64_t n = 0, nc = 0;
    double lam = 1.0;
};

// Work vectors of one V-cycle, one set per stream the PC is applied on (the
// concurrent 3-way block PC applies the same s/f PCs on two streams at once).
struct AmgWork {
    std::vector<DBuf<double>> r, d, x, b;  // per level; x, b unused on level 0
    DBuf<double> cx, cb;                   // coarsest level
};

struct PCAMG : PC {
    std::vector<std::unique_ptr<AmgLevel>> lv;
    int K = 2;
    int64_t nco = 0;
    DevCSR Cinv;                   // dense inverse of the coarsest operator
    std::unique_ptr<PC> Clu;       // ... or its device LU (dense inverse while it fits)
    std::unique_ptr<DevCSR> Cmat;
    std::map<hipStream_t, std::unique_ptr<AmgWork>> work;

    bool reentrant() const override { return true; }

    AmgWork &work_for(Ctx &c) {
        auto &w = work[c.st];
        if (!w) {
            w = std::make_unique<AmgWork>();
            const size_t L = lv.size();
            w->r.resize(L);
            w->d.resize(L);
            w->x.resize(L);
            w->b.resize(L);
            for (size_t l = 0; l < L; ++l) {
                const size_t m = (size_t)std::max<int64_t>(lv[l]->n, 1);
                w->r[l].alloc(m);
                w->d[l].alloc(m);
                if (l > 0) {
                    w->x[l].alloc(m);
                    w->b[l].alloc(m);
                }
            }
            w->cx.alloc(std::max<int64_t>(nco, 1));
            w->cb.alloc(std::max<int64_t>(nco, 1));
        }
        return *w;
    }

    PCAMG(const DevCSR &M, const Options &o, const std::string &prefix, bool hypre, Ctx &c) {
        type = hypre ? "hypre" : "gamg";
        n = M.nrows;
        const double theta = o.num(prefix + "pc_gamg_threshold", 0.0);
        const int64_t limit = o.integer(prefix + "pc_gamg_coarse_eq_limit", 50);
        const int64_t maxlev = o.integer(prefix + "pc_mg_levels", 10);
        // smoothing steps: PCMG's level KSP max_it; the hypre stand-in reads
        // BoomerAMG's sweep count (reference petsc-options-inexact: 1)
        const int64_t kdef = hypre ? o.integer(prefix + "pc_hypre_boomeramg_grid_sweeps_all", 1) : 2;
        K = (int)o.integer(prefix + "mg_levels_ksp_max_it", kdef);
        if (K < 1) throw Error(prefix + "mg_levels_ksp_max_it must be >= 1");
        if (!M.sell) build_sell(const_cast<DevCSR &>(M), c);
        const bool view = o.flag("pls.amg_view", false);
        double tm[8] = {0};  // setup stage seconds (pls.amg_view)
        auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
        double t0 = now();
        HostCSR A = download(M, c);
        tm[0] += now() - t0;
        std::unique_ptr<DevCSR> cur;  // device copy of A on levels > 0
        while (A.nrows > limit && (int64_t)lv.size() < maxlev - 1) {
            int32_t na = 0;
            t0 = now();
            const std::vector<int32_t> agg = aggregate(A, theta, na);
            tm[1] += now() - t0;
            if (na >= A.nrows || na == 0) break;
            auto L = std::make_unique<AmgLevel>();
            L->n = A.nrows;
            L->nc = na;
            std::vector<int64_t> sz(na, 0);
            for (int32_t a : agg) ++sz[a];
            HostCSR P0;
            P0.nrows = A.nrows;
            P0.ncols = na;
            P0.rp.resize(A.nrows + 1);
            P0.ci.resize(A.nrows);
            P0.v.resize(A.nrows);
            P0.rp[0] = 0;
            for (int64_t i = 0; i < A.nrows; ++i) {
                P0.rp[i + 1] = i + 1;
                P0.ci[i] = agg[i];
                P0.v[i] = 1.0 / std::sqrt((double)sz[agg[i]]);
            }
            const std::vector<double> dinv = jacobi_dinv(A);
            t0 = now();
            L->lam = power_lambda(A, dinv, 15);
            tm[2] += now() - t0;
            t0 = now();
            const double omega = 4.0 / (3.0 * L->lam);
            const HostCSR AP0 = spgemm(A, P0);
            HostCSR P;  // P0 - omega (D^-1 A P0), merged row by row (csr_binop)
            P.nrows = A.nrows;
            P.ncols = na;
            auto put = [&P](int32_t j, double v) {
                if (v != 0.0) {
                    P.ci.push_back(j);
                    P.v.push_back(v);
                }
            };
            for (int64_t i = 0; i < A.nrows; ++i) {
                const int32_t j0 = P0.ci[i];
                bool done0 = false;
                for (int64_t k = AP0.rp[i]; k < AP0.rp[i + 1]; ++k) {
                    const int32_t j = AP0.ci[k];
                    const double s = omega * (dinv[i] * AP0.v[k]);
                    if (!done0 && j0 < j) {
                        put(j0, P0.v[i] - 0.0);
                        done0 = true;
                    }
                    if (j == j0) {
                        put(j, P0.v[i] - s);
                        done0 = true;
                    } else {
                        put(j, 0.0 - s);
                    }
                }
                if (!done0) put(j0, P0.v[i] - 0.0);
                P.rp.push_back((int64_t)P.ci.size());
            }
            const HostCSR R = transpose(P);
            tm[3] += now() - t0;
            t0 = now();
            HostCSR Ac;
            if (!galerkin_fused(A, P, na, o.num("pls.amg_rap_dense_gb", 16.0) * 1e9, Ac)) Ac = spgemm(R, spgemm(A, P));
            tm[4] += now() - t0;
            t0 = now();
            L->Aown = std::move(cur);
            L->A = L->Aown ? L->Aown.get() : &M;
            L->dinv.alloc(std::max<int64_t>(A.nrows, 1));
            HIPCHK(hipMemcpyAsync(L->dinv.p, dinv.data(), sizeof(double) * A.nrows, hipMemcpyHostToDevice, c.st));
            upload(P, L->P, c);
            upload(R, L->R, c);
            amg_layout(L->P, c);
            amg_layout(L->R, c);
            lv.push_back(std::move(L));
            cur = std::make_unique<DevCSR>();
            upload(Ac, *cur, c);
            amg_layout(*cur, c);
            A = std::move(Ac);
            c.sync();
            tm[5] += now() - t0;
        }
        nco = A.nrows;
        work_for(c);
        if (nco > 0) {
            if (nco <= 1024) {
                upload(dense_inverse(A), Cinv, c);
                amg_layout(Cinv, c);
            } else {
                Cmat = std::move(cur);
                const DevCSR &Cm = Cmat ? *Cmat : M;
                if (nco <= o.integer("pls.lu_dense_max", 32768)) Clu = std::make_unique<PCDenseLU>(Cm, c);
                else Clu = std::make_unique<PCILU>(Cm, 1, c, true, o.flag("pls.ilu_lds", true));
            }
        }
        c.sync();
        if (view) {
            fprintf(stderr, "[amg %s] levels %zu:", prefix.c_str(), lv.size() + 1);
            for (auto &L : lv) fprintf(stderr, " %lld(lam %.6g)", (long long)L->n, L->lam);
            fprintf(stderr, " coarse %lld\n", (long long)nco);
            fprintf(stderr,
                    "[amg %s] setup s: download %.2f aggregate %.2f lambda %.2f P/R %.2f RAP %.2f upload %.2f "
                    "(%d threads)\n",
                    prefix.c_str(), tm[0], tm[1], tm[2], tm[3], tm[4], tm[5], setup_threads());
        }
    }

    // K Chebyshev steps on level L from x (x_zero: x == 0 on entry, r = b)
    void smooth(size_t l, AmgWork &W, const double *b, double *x, bool x_zero, Ctx &c) {
        const AmgLevel &L = *lv[l];
        double *rw = W.r[l].p, *dw = W.d[l].p;
        const double lmax = 1.1 * L.lam, lmin = 0.1 * L.lam;
        const double th = (lmax + lmin) / 2.0, de = (lmax - lmin) / 2.0;
        const double sigma = th / de;
        double rho = 1.0 / sigma;
        const double *r = b;
        if (!x_zero) {
            spmv(*L.A, x, rw, c, -1.0, 1.0, b);
            r = rw;
        }
        launch_cheb_step(L.n, L.dinv.p, r, dw, x, 0.0, 1.0 / th, x_zero ? 3 : 1, c.st);
        for (int k = 1; k < K; ++k) {
            spmv(*L.A, x, rw, c, -1.0, 1.0, b);
            const double rn = 1.0 / (2.0 * sigma - rho);
            launch_cheb_step(L.n, L.dinv.p, rw, dw, x, rn * rho, 2.0 * rn / de, 0, c.st);
            rho = rn;
        }
    }

    void coarse_solve(const double *b, double *x, Ctx &c) {
        if (nco == 0) return;
        if (Clu) Clu->apply(b, x, c);
        else spmv(Cinv, b, x, c);
    }

    void vcycle(size_t l, AmgWork &W, const double *b, double *x, Ctx &c) {
        if (l == lv.size()) {
            coarse_solve(b, x, c);
            return;
        }
        const AmgLevel &L = *lv[l];
        const bool last = (l + 1 == lv.size());
        double *bc = last ? W.cb.p : W.b[l + 1].p;
        double *xc = last ? W.cx.p : W.x[l + 1].p;
        smooth(l, W, b, x, true, c);
        spmv(*L.A, x, W.r[l].p, c, -1.0, 1.0, b);
        spmv(L.R, W.r[l].p, bc, c);
        vcycle(l + 1, W, bc, xc, c);
        spmv(L.P, xc, x, c, 1.0, 1.0, x);
        smooth(l, W, b, x, false, c);
    }

    void apply(const double *x, double *y, Ctx &c) override {
        if (n == 0) return;
        if (lv.empty()) {
            coarse_solve(x, y, c);
            return;
        }
        vcycle(0, work_for(c), x, y, c);
    }
};

}  // namespace

std::unique_ptr<PC> make_amg(const DevCSR &M, const Options &o, const std::string &prefix, bool hypre, Ctx &c) {
    if (M.halo) throw Error("PC type gamg/hypre (prefix " + prefix + "): multigrid is single-rank in this build");
    return std::make_unique<PCAMG>(M, o, prefix, hypre, c);
}

}  // namespace pls
