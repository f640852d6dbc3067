// boomeramg.cpp -- classical algebraic multigrid as the reference configures
// hypre BoomerAMG (-X_pc_type hypre, petsc-options-inexact:16-24, :32-40,
// :48-56, :63-71, :92-100): strength of connection (strong_threshold,
// max_row_sum), HMIS coarsening (one rank: the Ruge-Stueben first pass),
// aggressive coarsening on the first agg_nl levels with agg_num_paths and
// multipass interpolation there, extended+i interpolation with P_max
// truncation elsewhere, Galerkin coarse operators, hybrid symmetric
// Gauss-Seidel smoothing (PCHYPRE's default relax type) in lexicographic
// (no_CF) or C/F order, Gaussian elimination on the coarsest level.
//
// The algorithm is specified in oracle/boomeramg.py (the test oracle); the
// setup here builds the same hierarchy bit for bit -- C/F splittings,
// interpolation weights and coarse operators -- by running every host sum in
// the order the spec writes it, without contraction.  Row-local stages
// (strength, S2, interpolation rows, truncation, Galerkin products) run on
// host threads (row results do not depend on the thread count); the
// coarsening pass is sequential by definition.  Smoothing is hypre's relax
// type 6 as its OpenMP build runs it with K threads (pls.hypre_relax_chunks,
// oracle "hybrid symmetric Gauss-Seidel with K chunks"): one symmetric sweep
// is x_I += M^-1 (b - A x)_I with M = (D + L) D^-1 (D + U) of the
// chunk-block-diagonal part, i.e. one ILU-style apply of the factors
// I + L D^-1 and D + U (PCILU in sgs mode) -- the chunks are its blocks, so
// one workgroup sweeps each chunk on libpls's level-scheduled LDS sweeps.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <map>
#include <memory>
#include <queue>
#include <thread>

#include "amg_host.hpp"
#include "kernels.hpp"

#pragma clang fp contract(off)

namespace pls {
namespace {
using namespace amgh;

struct Pattern {  // CSR sparsity (strong dependencies); arrays sized by their writers (hvec)
    int64_t n = 0;
    hvec<int64_t> rp{0};
    hvec<int32_t> ci;
    int64_t len(int64_t i) const { return rp[i + 1] - rp[i]; }
};

// concatenate per-thread pattern parts (rows in order); the parts are copied
// into place by their own threads (one serial copy of S was ~0.4 s at N=59)
Pattern concat_pattern(int64_t n, std::vector<Pattern> &part) {
    Pattern S;
    S.n = n;
    const size_t T = part.size();
    std::vector<int64_t> row0(T + 1, 0), nz0(T + 1, 0);
    for (size_t t = 0; t < T; ++t) {
        row0[t + 1] = row0[t] + (part[t].rp.empty() ? 0 : (int64_t)part[t].rp.size() - 1);
        nz0[t + 1] = nz0[t] + (int64_t)part[t].ci.size();
    }
    S.rp.assign(n + 1, 0);
    S.ci.resize(nz0[T]);
    std::vector<std::thread> th;
    for (size_t t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            Pattern &p = part[t];
            for (size_t k = 1; k < p.rp.size(); ++k) S.rp[row0[t] + k] = nz0[t] + p.rp[k];
            std::copy(p.ci.begin(), p.ci.end(), S.ci.begin() + nz0[t]);
            Pattern().rp.swap(p.rp);
            hvec<int32_t>().swap(p.ci);
        });
    for (auto &x : th) x.join();
    return S;
}

// oracle strength(): hypre CreateS with strong_threshold theta, max_row_sum mu.
// Two passes over the rows (threshold and count, then fill) into arrays sized
// once: per-thread push_back growth on GBs of output serialised the threads
// on page faults
Pattern strength(const HostCSR &A, double theta, double mu) {
    const int64_t n = A.nrows;
    const int T = setup_threads();
    Pattern S;
    S.n = n;
    S.rp.assign(n + 1, 0);
    std::vector<double> thr(n);
    std::vector<int8_t> mode(n);  // 0: no strong dependencies, 1: d >= 0 (a < thr), 2: d < 0 (a > thr)
    parallel_rows(n, T, [&](int, int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            double d = 0.0, rs = 0.0;
            double smin = std::numeric_limits<double>::infinity(), smax = -smin;
            int64_t noff = 0;
            for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                const double a = A.v[k];
                rs += a;
                if (A.ci[k] == i) {
                    d = a;
                } else {
                    ++noff;
                    smin = std::min(smin, a);
                    smax = std::max(smax, a);
                }
            }
            int64_t c = 0;
            mode[i] = 0;
            if (noff > 0 && !(mu < 1.0 && std::fabs(rs) > mu * std::fabs(d))) {
                const bool pos = d >= 0.0;
                const double t = theta * (pos ? smin : smax);
                thr[i] = t;
                mode[i] = pos ? 1 : 2;
                for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                    if (A.ci[k] == i) continue;
                    const double a = A.v[k];
                    c += pos ? a < t : a > t;
                }
            }
            S.rp[i + 1] = c;
        }
    });
    for (int64_t i = 0; i < n; ++i) S.rp[i + 1] += S.rp[i];
    S.ci.resize(S.rp[n]);
    parallel_rows(n, T, [&](int, int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            if (!mode[i]) continue;
            const bool pos = mode[i] == 1;
            const double t = thr[i];
            int64_t o = S.rp[i];
            for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                if (A.ci[k] == i) continue;
                const double a = A.v[k];
                if (pos ? a < t : a > t) S.ci[o++] = A.ci[k];
            }
        }
    });
    return S;
}

// S^T with every column's rows ascending (the sequential fill's order): per
// thread column counts over its row range, offsets thread-major inside each
// column, then every thread fills its rows -- memory-bound, on host threads
// (the sequential transpose was ~1.6 s of the N=40 s block's RS pass)
// (threads capped so the per-thread column counts, Tn x n, stay within nnz / 2
// entries; `max_threads` 1 inside an already parallel caller)
Pattern transpose(const Pattern &S, int max_threads = 0) {
    const int64_t n = S.n, nnz = (int64_t)S.ci.size();
    Pattern T;
    T.n = n;
    T.rp.assign(n + 1, 0);
    T.ci.resize(nnz);
    int Tn = max_threads > 0 ? std::min(max_threads, setup_threads()) : setup_threads();
    if (n > 0) Tn = (int)std::max<int64_t>(1, std::min<int64_t>(Tn, nnz / (2 * n)));
    if (nnz < (int64_t)1 << 20 || n < 1024) Tn = 1;
    if (Tn == 1) {
        for (int32_t j : S.ci) ++T.rp[j + 1];
        for (int64_t j = 0; j < n; ++j) T.rp[j + 1] += T.rp[j];
        std::vector<int64_t> pos(T.rp.begin(), T.rp.end() - 1);
        for (int64_t i = 0; i < n; ++i)
            for (int64_t k = S.rp[i]; k < S.rp[i + 1]; ++k) T.ci[pos[S.ci[k]]++] = (int32_t)i;
        return T;
    }
    std::vector<int64_t> r0(Tn + 1);
    for (int t = 0; t <= Tn; ++t) r0[t] = n * t / Tn;
    std::vector<std::vector<int64_t>> cnt(Tn);
    auto run = [&](auto fn) {
        std::vector<std::thread> th;
        for (int t = 0; t < Tn; ++t) th.emplace_back(fn, t);
        for (auto &x : th) x.join();
    };
    run([&](int t) {
        cnt[t].assign(n, 0);
        for (int64_t k = S.rp[r0[t]]; k < S.rp[r0[t + 1]]; ++k) ++cnt[t][S.ci[k]];
    });
    // column lengths, then per-thread starts inside each column (column ranges in parallel)
    run([&](int t) {
        for (int64_t j = r0[t]; j < r0[t + 1]; ++j) {
            int64_t c = 0;
            for (int q = 0; q < Tn; ++q) c += cnt[q][j];
            T.rp[j + 1] = c;
        }
    });
    for (int64_t j = 0; j < n; ++j) T.rp[j + 1] += T.rp[j];
    run([&](int t) {
        for (int64_t j = r0[t]; j < r0[t + 1]; ++j) {
            int64_t o = T.rp[j];
            for (int q = 0; q < Tn; ++q) {
                const int64_t c = cnt[q][j];
                cnt[q][j] = o;
                o += c;
            }
        }
    });
    run([&](int t) {
        std::vector<int64_t> &pos = cnt[t];
        for (int64_t i = r0[t]; i < r0[t + 1]; ++i)
            for (int64_t k = S.rp[i]; k < S.rp[i + 1]; ++k) T.ci[pos[S.ci[k]]++] = (int32_t)i;
    });
    return T;
}

constexpr int8_t UND = 0, FPT = -1, CPT = 1;

// oracle rs_first_pass(): HMIS on one rank.  The oracle's lazily updated heap
// selects argmax (lambda, -i) over the undecided points; here a tournament
// tree over the points holds that argmax (O(log n) per lambda change, no
// allocation), the same selection.
struct Tournament {
    int64_t size = 1;
    std::vector<int32_t> node;  // best point of each subtree, -1: none
    const std::vector<int64_t> &lam;
    const std::vector<int8_t> &st;
    Tournament(int64_t n, const std::vector<int64_t> &l, const std::vector<int8_t> &s) : lam(l), st(s) {
        while (size < n) size <<= 1;
        node.assign(2 * size, -1);
        for (int64_t i = 0; i < n; ++i) node[size + i] = s[i] == 0 ? (int32_t)i : -1;
        for (int64_t v = size - 1; v >= 1; --v) node[v] = better(node[2 * v], node[2 * v + 1]);
    }
    int32_t better(int32_t a, int32_t b) const {
        if (a < 0) return b;
        if (b < 0) return a;
        if (lam[a] != lam[b]) return lam[a] > lam[b] ? a : b;
        return a < b ? a : b;
    }
    void update(int64_t i) {  // after lam[i] or st[i] changed
        int64_t v = size + i;
        node[v] = st[i] == 0 ? (int32_t)i : -1;
        for (v >>= 1; v >= 1; v >>= 1) {
            const int32_t b = better(node[2 * v], node[2 * v + 1]);
            if (node[v] == b && b != (int32_t)i) break;  // unchanged above
            node[v] = b;
        }
    }
};

// The same argmax by groups (round 4; round 3 kept a per-point bitmap per
// lambda bucket): the points in groups of 64, each
// group's largest lambda over its undecided points kept in gmax, and the
// groups in lambda buckets (a two-level bitmap per bucket over the groups:
// ~1 MB at 2.5M points, where a per-point bitmap per bucket was ~50 MB and
// every lambda change a DRAM access).  A lambda change rescans its group's 64
// lambdas only when it lowers the group's maximum; a selection takes the top
// bucket's first group and that group's first point at the top lambda --
// the largest lambda, ties to the smallest index, as before.
struct GroupMax {
    const hvec<int32_t> &lk;
    int64_t n, ng, w1, w2, NB, top = -1;
    std::vector<int32_t> gmax;
    std::vector<uint64_t> b0, b1;
    std::vector<int64_t> cnt;
    GroupMax(const hvec<int32_t> &l, int64_t n_, int64_t maxlam) : lk(l), n(n_) {
        ng = (n + 63) / 64;
        w1 = (ng + 63) / 64;
        w2 = (w1 + 63) / 64;
        NB = maxlam + 1;
        gmax.assign(ng, -1);
        b0.assign((size_t)(NB * w1), 0);
        b1.assign((size_t)(NB * w2), 0);
        cnt.assign(NB, 0);
        for (int64_t g = 0; g < ng; ++g) {
            gmax[g] = scan(g);
            if (gmax[g] >= 0) insert(gmax[g], g);
        }
    }
    int32_t scan(int64_t g) const {
        int32_t m = -1;
        const int64_t e = std::min(n, (g + 1) * 64);
        for (int64_t i = g * 64; i < e; ++i) m = std::max(m, lk[i]);
        return m;
    }
    void insert(int64_t v, int64_t g) {
        uint64_t &x = b0[v * w1 + (g >> 6)];
        if (!x) b1[v * w2 + (g >> 12)] |= 1ull << ((g >> 6) & 63);
        x |= 1ull << (g & 63);
        ++cnt[v];
        if (v > top) top = v;
    }
    void erase(int64_t v, int64_t g) {
        uint64_t &x = b0[v * w1 + (g >> 6)];
        x &= ~(1ull << (g & 63));
        if (!x) b1[v * w2 + (g >> 12)] &= ~(1ull << ((g >> 6) & 63));
        --cnt[v];
    }
    // lk[i] went from oldv to newv (-1: decided)
    void changed(int64_t i, int32_t oldv, int32_t newv) {
        const int64_t g = i >> 6;
        const int32_t m = gmax[g];
        if (newv > m) {
            if (m >= 0) erase(m, g);
            gmax[g] = newv;
            insert(newv, g);
        } else if (oldv == m && newv < oldv) {
            const int32_t nm = scan(g);
            if (nm != m) {
                erase(m, g);
                gmax[g] = nm;
                if (nm >= 0) insert(nm, g);
            }
        }
    }
    int64_t best() {
        while (top >= 0 && cnt[top] == 0) --top;
        if (top < 0) return -1;
        int64_t k1 = 0;
        while (!b1[top * w2 + k1]) ++k1;
        const int64_t k0 = (k1 << 6) | __builtin_ctzll(b1[top * w2 + k1]);
        const int64_t g = (k0 << 6) | __builtin_ctzll(b0[top * w1 + k0]);
        for (int64_t i = g * 64;; ++i)
            if (lk[i] == top) return i;
    }
};

std::vector<int8_t> rs_first_pass(const Pattern &S, int max_threads = 0) {
    const int64_t n = S.n;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t0 = now();
    const Pattern ST = transpose(S, max_threads);
    const double t1 = now();
    std::vector<int64_t> lam(n);
    int64_t maxst = 0;
    for (int64_t i = 0; i < n; ++i) {
        lam[i] = ST.len(i);
        maxst = std::max(maxst, lam[i]);
    }
    std::vector<int8_t> st(n, UND);
    for (int64_t i = 0; i < n; ++i)
        if (S.len(i) == 0 && lam[i] == 0) st[i] = FPT;
    // prepass: undecided points with lambda 0 become F in ascending order
    // (their dependencies' lambda grow, possibly above 0 before their turn)
    for (int64_t j = 0; j < n; ++j) {
        if (st[j] != UND || lam[j] != 0) continue;
        st[j] = FPT;
        for (int64_t q = S.rp[j]; q < S.rp[j + 1]; ++q)
            if (st[S.ci[q]] == UND) ++lam[S.ci[q]];
    }
    if (std::getenv("PLS_RS_TOURNAMENT")) {  // (the round-2 selection structure; same result)
        Tournament T(n, lam, st);
        auto make_f = [&](int64_t j) {
            st[j] = FPT;
            T.update(j);
            for (int64_t q = S.rp[j]; q < S.rp[j + 1]; ++q) {
                const int32_t k = S.ci[q];
                if (st[k] == UND) {
                    ++lam[k];
                    T.update(k);
                }
            }
        };
        while (T.node[1] >= 0) {
            const int64_t i = T.node[1];
            st[i] = CPT;
            T.update(i);
            for (int64_t q = ST.rp[i]; q < ST.rp[i + 1]; ++q)
                if (st[ST.ci[q]] == UND) make_f(ST.ci[q]);
            for (int64_t q = S.rp[i]; q < S.rp[i + 1]; ++q) {
                const int32_t k = S.ci[q];
                if (st[k] != UND) continue;
                if (--lam[k] == 0) make_f(k);
                else T.update(k);
            }
        }
    } else {
        // lk: lambda of an undecided point, -1 once decided (one int32 array:
        // one random access per neighbour instead of state + lambda)
        hvec<int32_t> lk(n);
        for (int64_t i = 0; i < n; ++i) lk[i] = st[i] == UND ? (int32_t)lam[i] : -1;
        GroupMax B(lk, n, 2 * maxst + 1);
        auto make_f = [&](int64_t j) {  // j undecided
            st[j] = FPT;
            const int32_t o = lk[j];
            lk[j] = -1;
            B.changed(j, o, -1);
            for (int64_t q = S.rp[j]; q < S.rp[j + 1]; ++q) {
                const int32_t k = S.ci[q];
                if (lk[k] >= 0) {
                    ++lk[k];
                    B.changed(k, lk[k] - 1, lk[k]);
                }
            }
        };
        for (int64_t i; (i = B.best()) >= 0;) {
            st[i] = CPT;
            const int32_t o = lk[i];
            lk[i] = -1;
            B.changed(i, o, -1);
            for (int64_t q = ST.rp[i]; q < ST.rp[i + 1]; ++q)
                if (lk[ST.ci[q]] >= 0) make_f(ST.ci[q]);
            for (int64_t q = S.rp[i]; q < S.rp[i + 1]; ++q) {
                const int32_t k = S.ci[q];
                if (lk[k] < 0) continue;
                --lk[k];
                B.changed(k, lk[k] + 1, lk[k]);
                if (lk[k] == 0) make_f(k);
            }
        }
    }
    for (auto &s : st)
        if (s == UND) s = FPT;
    if (std::getenv("PLS_AMG_TRACE") && n > 100000)
        fprintf(stderr, "[rs_first_pass] n %lld: transpose %.2f s, pass %.2f s\n", (long long)n, t1 - t0, now() - t1);
    return st;
}

// oracle second_strength(): S2 over the C points (local numbering)
Pattern second_strength(const Pattern &S, const std::vector<int8_t> &cf, int paths, std::vector<int32_t> &cpts) {
    const int64_t n = S.n;
    std::vector<int32_t> loc(n, -1);
    cpts.clear();
    for (int64_t i = 0; i < n; ++i)
        if (cf[i] == CPT) {
            loc[i] = (int32_t)cpts.size();
            cpts.push_back((int32_t)i);
        }
    const int64_t m = (int64_t)cpts.size();
    const int T = setup_threads();
    // SC: every row of S restricted to the C1 points, in C1 numbering -- the
    // path counts then run over ~1/10 of S's entries with an m-sized counter
    Pattern SC;
    SC.n = n;
    SC.rp.assign(n + 1, 0);
    parallel_rows(n, T, [&](int, int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            int64_t c = 0;
            for (int64_t q = S.rp[i]; q < S.rp[i + 1]; ++q) c += loc[S.ci[q]] >= 0;
            SC.rp[i + 1] = c;
        }
    });
    for (int64_t i = 0; i < n; ++i) SC.rp[i + 1] += SC.rp[i];
    SC.ci.resize(SC.rp[n]);
    parallel_rows(n, T, [&](int, int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            int64_t o = SC.rp[i];
            for (int64_t q = S.rp[i]; q < S.rp[i + 1]; ++q)
                if (loc[S.ci[q]] >= 0) SC.ci[o++] = loc[S.ci[q]];
        }
    });
    std::vector<Pattern> part(T);
    parallel_rows(m, T, [&](int t, int64_t c0, int64_t c1) {
        Pattern &P = part[t];
        P.rp.assign(1, 0);
        std::vector<int32_t> cnt(m, 0), tbuf(m + 1), row;
        for (int64_t c = c0; c < c1; ++c) {
            const int64_t i = cpts[c];
            int64_t nt = 0;
            auto bump_row = [&](int64_t k) {
                for (int64_t r = SC.rp[k]; r < SC.rp[k + 1]; ++r) {
                    const int32_t j = SC.ci[r];
                    tbuf[nt] = j;
                    nt += (cnt[j] == 0) & (j != c);
                    cnt[j] += j != c;
                }
            };
            bump_row(i);
            for (int64_t q = S.rp[i]; q < S.rp[i + 1]; ++q) bump_row(S.ci[q]);
            row.clear();
            for (int64_t u = 0; u < nt; ++u) {
                const int32_t j = tbuf[u];
                if (cnt[j] >= paths) row.push_back(j);
                cnt[j] = 0;
            }
            std::sort(row.begin(), row.end());
            P.ci.insert(P.ci.end(), row.begin(), row.end());
            P.rp.push_back((int64_t)P.ci.size());
        }
    });
    return concat_pattern(m, part);
}

// oracle rs_partitioned(): the first pass inside each of K contiguous
// partitions (hypre's ChunkMap sizes over S.n; `pt` maps a point to its
// position in the partitioned set when S is a subset, e.g. the C1 points) on
// the strong connections inside it; partitions run on host threads.
std::vector<int8_t> rs_partitioned(const Pattern &S, int64_t K, const std::vector<int64_t> &part_start) {
    const int64_t n = S.n;
    if (K <= 1 || n == 0) return rs_first_pass(S);
    std::vector<int8_t> cf(n, FPT);
    // partitions on host threads; with fewer partitions than threads each
    // partition's extraction and transpose get the spare threads
    const int T = setup_threads();
    const int Tk = (int)std::max<int64_t>(1, T / K);
    auto nowp = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double ts = nowp();
    // (threads over partitions directly: parallel_rows keeps >= 8 items per thread)
    const int Tp = (int)std::min<int64_t>(K, T);
    std::vector<std::thread> pool;
    for (int t = 0; t < Tp; ++t) pool.emplace_back([&, t] {
        for (int64_t k = K * t / Tp; k < K * (t + 1) / Tp; ++k) {
            const int64_t a = part_start[k], b = part_start[k + 1];
            if (b <= a) continue;
            Pattern L;
            L.n = b - a;
            L.rp.assign(L.n + 1, 0);
            auto inside = [&](int32_t j) { return j >= a && j < b; };
            parallel_rows(L.n, Tk, [&](int, int64_t i0, int64_t i1) {
                for (int64_t i = i0; i < i1; ++i) {
                    int64_t c = 0;
                    for (int64_t q = S.rp[a + i]; q < S.rp[a + i + 1]; ++q) c += inside(S.ci[q]);
                    L.rp[i + 1] = c;
                }
            });
            for (int64_t i = 0; i < L.n; ++i) L.rp[i + 1] += L.rp[i];
            L.ci.resize(L.rp[L.n]);
            parallel_rows(L.n, Tk, [&](int, int64_t i0, int64_t i1) {
                for (int64_t i = i0; i < i1; ++i) {
                    int64_t o = L.rp[i];
                    for (int64_t q = S.rp[a + i]; q < S.rp[a + i + 1]; ++q)
                        if (inside(S.ci[q])) L.ci[o++] = (int32_t)(S.ci[q] - a);
                }
            });
            const double tx = nowp();
            const std::vector<int8_t> lc = rs_first_pass(L, Tk);
            if (std::getenv("PLS_AMG_TRACE"))
                fprintf(stderr, "[rs_partitioned] part %lld: extracted %.3f, passed %.3f s\n", (long long)k, tx - ts, nowp() - ts);
            std::copy(lc.begin(), lc.end(), cf.begin() + a);
        }
    });
    for (auto &x : pool) x.join();
    return cf;
}

// oracle coarsen_partition(): the most partitions (<= K, halving) whose
// boundaries cut at most 2 % of the strong connections; 1 if none does
int64_t coarsen_partitions(const Pattern &S, int64_t K) {
    const int64_t n = S.n, nnz = (int64_t)S.ci.size();
    while (K > 1) {
        const int64_t q = n / K, r = n % K;
        auto part = [&](int64_t i) { return i < r * (q + 1) ? i / (q + 1) : r + (i - r * (q + 1)) / q; };
        const int T = setup_threads();
        std::vector<int64_t> cuts(T, 0);
        parallel_rows(n, T, [&](int t, int64_t i0, int64_t i1) {
            int64_t c = 0;
            for (int64_t i = i0; i < i1; ++i) {
                const int64_t pi = part(i);
                for (int64_t k = S.rp[i]; k < S.rp[i + 1]; ++k) c += pi != part(S.ci[k]);
            }
            cuts[t] = c;
        });
        int64_t cut = 0;
        for (int64_t c : cuts) cut += c;
        if (nnz == 0 || cut <= 0.02 * (double)nnz) return K;
        K /= 2;
    }
    return 1;
}

// partition starts of n points in K chunks (hypre's thread partition)
std::vector<int64_t> chunk_starts(int64_t n, int64_t K) {
    std::vector<int64_t> st(K + 1, 0);
    const int64_t q = n / K, r = n % K;
    for (int64_t k = 0; k < K; ++k) st[k + 1] = st[k] + q + (k < r ? 1 : 0);
    return st;
}

// oracle hypre_rand(): hypre_Rand() after hypre_SeedRand(seed), Park-Miller by Schrage
struct HypreRand {
    int64_t s;
    explicit HypreRand(int64_t seed) : s(seed) {}
    double next() {
        const int64_t hi = s / 127773, lo = s % 127773;
        const int64_t t = 16807 * lo - 2836 * hi;
        s = t > 0 ? t : t + 2147483647;
        return (double)s / 2147483647.0;
    }
};

// oracle pmis_stage(): HMIS's PMIS stage over the first pass's splitting
// (partition k = process k: seeds 2747 + k; boundary = a strong dependency on
// another partition's point)
std::vector<int8_t> pmis_stage(const Pattern &S, const std::vector<int8_t> &cf1, const std::vector<int64_t> &pst) {
    const int64_t n = S.n;
    if (n == 0 || pst.size() <= 2) return cf1;  // one partition: no boundary points
    const int64_t K = (int64_t)pst.size() - 1;
    const int T = setup_threads();
    std::vector<int32_t> part(n, 0);
    for (int64_t k = 0; k < K; ++k) std::fill(part.begin() + pst[k], part.begin() + pst[k + 1], (int32_t)k);
    // boundary points (the only ones PMIS decides; the rest keep the first pass's marker)
    std::vector<int32_t> bidx(n, -1);
    std::vector<std::vector<int32_t>> bl(T);
    parallel_rows(n, T, [&](int t, int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            bool boundary = false;
            for (int64_t q = S.rp[i]; q < S.rp[i + 1] && !boundary; ++q) boundary = part[S.ci[q]] != part[i];
            if (boundary) bl[t].push_back((int32_t)i);
        }
    });
    std::vector<int32_t> B;
    for (auto &v : bl) B.insert(B.end(), v.begin(), v.end());
    const int64_t nb = (int64_t)B.size();
    for (int64_t b = 0; b < nb; ++b) bidx[B[b]] = (int32_t)b;
    // S^T restricted to the boundary points' rows: per thread, the entries j -> i
    // (i a boundary point) of its row range, then merged in row order
    std::vector<std::vector<std::pair<int32_t, int32_t>>> te(T);
    parallel_rows(n, T, [&](int t, int64_t j0, int64_t j1) {
        for (int64_t j = j0; j < j1; ++j)
            for (int64_t q = S.rp[j]; q < S.rp[j + 1]; ++q)
                if (bidx[S.ci[q]] >= 0) te[t].emplace_back(bidx[S.ci[q]], (int32_t)j);
    });
    std::vector<int64_t> trp(nb + 1, 0);
    for (auto &v : te)
        for (auto &e : v) ++trp[e.first + 1];
    for (int64_t b = 0; b < nb; ++b) trp[b + 1] += trp[b];
    std::vector<int32_t> tci(trp[nb]);
    {
        std::vector<int64_t> pos(trp.begin(), trp.end() - 1);
        for (auto &v : te)  // threads in row order: every S^T row ascending
            for (auto &e : v) tci[pos[e.first]++] = e.second;
    }
    std::vector<double> measure(n);
    for (int64_t k = 0; k < K; ++k) {
        HypreRand r(2747 + k);
        for (int64_t i = pst[k]; i < pst[k + 1]; ++i) {
            const double u = r.next();
            measure[i] = bidx[i] >= 0 ? (double)(trp[bidx[i] + 1] - trp[bidx[i]]) + u : 0.0;
        }
    }
    std::vector<int8_t> st(cf1);
    for (int64_t b = 0; b < nb; ++b) st[B[b]] = trp[b + 1] == trp[b] ? FPT : UND;
    std::vector<int8_t> nxt(nb);
    auto apply = [&]() {
        for (int64_t b = 0; b < nb; ++b) st[B[b]] = nxt[b];
    };
    auto mark_f = [&]() {  // undecided points with a strong dependency on a C point -> F
        std::vector<int64_t> und(T, 0);
        parallel_rows(nb, T, [&](int t, int64_t b0, int64_t b1) {
            for (int64_t b = b0; b < b1; ++b) {
                const int64_t i = B[b];
                int8_t s = st[i];
                if (s == UND) {
                    for (int64_t q = S.rp[i]; q < S.rp[i + 1]; ++q)
                        if (st[S.ci[q]] == CPT) {
                            s = FPT;
                            break;
                        }
                    und[t] += s == UND;
                }
                nxt[b] = s;
            }
        });
        apply();
        int64_t u = 0;
        for (int64_t x : und) u += x;
        return u;
    };
    for (int64_t left = mark_f(); left > 0; left = mark_f()) {
        std::vector<int64_t> sel(T, 0);
        parallel_rows(nb, T, [&](int t, int64_t b0, int64_t b1) {
            for (int64_t b = b0; b < b1; ++b) {
                const int64_t i = B[b];
                int8_t s = st[i];
                if (s == UND) {
                    bool best = true;
                    const double mi = measure[i];
                    for (int64_t q = S.rp[i]; q < S.rp[i + 1] && best; ++q)
                        best = st[S.ci[q]] != UND || mi > measure[S.ci[q]];
                    for (int64_t q = trp[b]; q < trp[b + 1] && best; ++q) best = st[tci[q]] != UND || mi > measure[tci[q]];
                    if (best) {
                        s = CPT;
                        ++sel[t];
                    }
                }
                nxt[b] = s;
            }
        });
        apply();
        int64_t ns = 0;
        for (int64_t x : sel) ns += x;
        if (ns == 0) {  // (the oracle's guard: ties of measures)
            int64_t bb = -1;
            for (int64_t b = 0; b < nb; ++b)
                if (st[B[b]] == UND && (bb < 0 || measure[B[b]] > measure[B[bb]])) bb = b;
            st[B[bb]] = CPT;
        }
    }
    for (auto &x : st)
        if (x != CPT) x = FPT;
    return st;
}

std::vector<int8_t> coarsen(const Pattern &S, bool aggressive, int paths, const std::vector<int64_t> &pst) {
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double t0 = now();
    const int64_t K = (int64_t)pst.size() - 1;
    std::vector<int8_t> cf = rs_partitioned(S, K, pst);
    const double tr = now();
    cf = pmis_stage(S, cf, pst);
    if (std::getenv("PLS_AMG_TRACE"))
        fprintf(stderr, "[boomeramg coarsen] n %lld K %lld: first pass %.2f s, PMIS stage %.2f s\n", (long long)S.n,
                (long long)K, tr - t0, now() - tr);
    if (!aggressive) return cf;
    double t1 = now();
    std::vector<int32_t> cpts;
    const Pattern S2 = second_strength(S, cf, paths, cpts);
    double t2 = now();
    // the C1 points' partitions: positions in cpts where the original chunk changes
    std::vector<int64_t> pst2(K + 1, 0);
    {
        size_t t = 0;
        for (int64_t k = 0; k < K; ++k) {
            pst2[k] = (int64_t)t;
            while (t < cpts.size() && cpts[t] < pst[k + 1]) ++t;
        }
        pst2[K] = (int64_t)cpts.size();
    }
    // (K: partitions, some possibly empty)
    const std::vector<int8_t> cf2 = pmis_stage(S2, rs_partitioned(S2, K, pst2), pst2);
    if (std::getenv("PLS_AMG_TRACE"))
        fprintf(stderr, "[boomeramg coarsen] n %lld S nnz %lld: RS %.2f s; S2 (%zu C1 points, nnz %lld) %.2f s; RS2 %.2f s\n",
                (long long)S.n, (long long)S.ci.size(), t1 - t0, cpts.size(), (long long)S2.ci.size(), t2 - t1, now() - t2);
    std::vector<int8_t> out(S.n, FPT);
    for (size_t c = 0; c < cpts.size(); ++c)
        if (cf2[c] == CPT) out[cpts[c]] = CPT;
    return out;
}

// rows (sorted column, value) -> HostCSR; exact zeros dropped
struct RowSet {
    std::vector<std::vector<int32_t>> col;
    std::vector<std::vector<double>> val;
};
HostCSR to_csr(RowSet &R, int64_t ncols) {  // (R's rows are released)
    HostCSR P;
    const int64_t n = (int64_t)R.col.size();
    P.nrows = n;
    P.ncols = ncols;
    P.rp.assign(n + 1, 0);
    const int T = setup_threads();
    parallel_rows(n, T, [&](int, int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            int64_t c = 0;
            for (double x : R.val[i]) c += x != 0.0;
            P.rp[i + 1] = c;
        }
    });
    for (int64_t i = 0; i < n; ++i) P.rp[i + 1] += P.rp[i];
    P.ci.resize(P.rp[n]);
    P.v.resize(P.rp[n]);
    parallel_rows(n, T, [&](int, int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            int64_t o = P.rp[i];
            for (size_t k = 0; k < R.col[i].size(); ++k)
                if (R.val[i][k] != 0.0) {
                    P.ci[o] = R.col[i][k];
                    P.v[o++] = R.val[i][k];
                }
            std::vector<int32_t>().swap(R.col[i]);
            std::vector<double>().swap(R.val[i]);
        }
    });
    return P;
}

// dense accumulator of one thread: first-touch order kept, sorted on output
struct Acc {  // sparse accumulator: v is all zero between rows, the touched list grows branch-free
    std::vector<double> v;
    std::vector<uint8_t> on;
    std::vector<int32_t> buf;
    int64_t cnt = 0;
    explicit Acc(int64_t n) : v(n, 0.0), on(n, 0), buf(n + 1) {}
    void add(int32_t j, double x) {
        buf[cnt] = j;
        cnt += on[j] ^ 1;
        on[j] = 1;
        v[j] += x;
    }
    int32_t *begin() { return buf.data(); }
    int32_t *end() { return buf.data() + cnt; }
    void sort() { std::sort(begin(), end()); }
    void clear() {
        for (int64_t u = 0; u < cnt; ++u) {
            on[buf[u]] = 0;
            v[buf[u]] = 0.0;
        }
        cnt = 0;
    }
};

std::vector<int32_t> coarse_index(const std::vector<int8_t> &cf, int64_t &nc) {
    std::vector<int32_t> ci(cf.size(), -1);
    nc = 0;
    for (size_t i = 0; i < cf.size(); ++i)
        if (cf[i] == CPT) ci[i] = (int32_t)nc++;
    return ci;
}

// oracle multipass_interp().  Rows live in per-thread arenas of fixed-size
// blocks (a row never straddles blocks, so its pointers stay valid while later
// passes read it); C rows point at cidx and a 1.0 -- no per-row allocations
// (5M std::vector rows were ~10M mallocs and a serial 240 MB init at N=59).
HostCSR multipass(const HostCSR &A, const Pattern &S, const std::vector<int8_t> &cf) {
    const int64_t n = A.nrows;
    int64_t nc = 0;
    const std::vector<int32_t> cidx = coarse_index(cf, nc);
    std::vector<int32_t> pass(n, -1);
    for (int64_t i = 0; i < n; ++i)
        if (cf[i] == CPT) pass[i] = 0;
    struct RowRef {
        const int32_t *c;
        const double *v;
        int64_t len;
    };
    static const double one = 1.0;
    hvec<RowRef> ref(n);
    for (int64_t i = 0; i < n; ++i) ref[i] = cf[i] == CPT ? RowRef{&cidx[i], &one, 1} : RowRef{nullptr, nullptr, 0};
    struct Arena {
        const int64_t BLK = (int64_t)1 << 18;
        std::vector<std::unique_ptr<int32_t[]>> cb;
        std::vector<std::unique_ptr<double[]>> vb;
        int64_t used = 0, cap = 0;
        void room(int64_t m) {  // m entries contiguous
            if (used + m <= cap) return;
            cap = std::max(BLK, m);
            cb.emplace_back(new int32_t[cap]);
            vb.emplace_back(new double[cap]);
            used = 0;
        }
    };
    const int T = setup_threads();
    struct State {
        Acc acc;
        std::vector<int32_t> Q;
        std::vector<double> aq;
        Arena ar;
        explicit State(int64_t nc) : acc(nc) {}
    };
    std::vector<std::unique_ptr<State>> state(T);
    for (int t = 0; t < T; ++t) state[t] = std::make_unique<State>(nc);
    for (int p = 1;; ++p) {
        // the points of pass p, decided from the passes before p (rows in parallel, kept in order)
        std::vector<std::vector<int32_t>> found(T);
        parallel_rows(n, T, [&](int t, int64_t i0, int64_t i1) {
            for (int64_t i = i0; i < i1; ++i) {
                if (pass[i] >= 0) continue;
                for (int64_t q = S.rp[i]; q < S.rp[i + 1]; ++q) {
                    const int32_t k = S.ci[q];
                    if (pass[k] >= 0 && pass[k] < p) {
                        found[t].push_back((int32_t)i);
                        break;
                    }
                }
            }
        });
        std::vector<int32_t> pts;
        for (auto &f : found) pts.insert(pts.end(), f.begin(), f.end());
        if (std::getenv("PLS_AMG_TRACE") && n > 100000) fprintf(stderr, "[multipass] pass %d: %zu points\n", p, pts.size());
        if (pts.empty()) break;
        for (int32_t i : pts) pass[i] = p;
        parallel_dynamic((int64_t)pts.size(), T, 256, [](int) {}, [&](int th, int64_t t0, int64_t t1) {
            State &X = *state[th];
            Acc &acc = X.acc;
            std::vector<int32_t> &Q = X.Q;
            std::vector<double> &aq = X.aq;
            for (int64_t t = t0; t < t1; ++t) {
                const int64_t i = pts[t];
                Q.clear();
                aq.clear();
                for (int64_t q = S.rp[i]; q < S.rp[i + 1]; ++q) {
                    const int32_t k = S.ci[q];
                    if (pass[k] >= 0 && pass[k] < p) Q.push_back(k);
                }
                double d = 0.0, neg_all = 0.0, pos_all = 0.0, neg_q = 0.0, pos_q = 0.0;
                size_t qi = 0;
                aq.assign(Q.size(), 0.0);
                for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                    const int32_t j = A.ci[k];
                    const double a = A.v[k];
                    if (j == i) {
                        d = a;
                        continue;
                    }
                    neg_all += std::min(a, 0.0);
                    pos_all += std::max(a, 0.0);
                    while (qi < Q.size() && Q[qi] < j) ++qi;
                    if (qi < Q.size() && Q[qi] == j) aq[qi] = a;
                }
                for (size_t u = 0; u < Q.size(); ++u) {
                    neg_q += std::min(aq[u], 0.0);
                    pos_q += std::max(aq[u], 0.0);
                }
                double alpha = 0.0, beta = 0.0;
                if (neg_q == 0.0) d += neg_all;
                else alpha = neg_all / neg_q;
                if (pos_q == 0.0) d += pos_all;
                else beta = pos_all / pos_q;
                for (size_t u = 0; u < Q.size(); ++u) {
                    const double a = aq[u];
                    if (a == 0.0) continue;
                    const double w = -(a < 0.0 ? alpha : beta) * a / d;
                    const RowRef &r = ref[Q[u]];
                    for (int64_t e = 0; e < r.len; ++e) acc.add(r.c[e], w * r.v[e]);
                }
                acc.sort();
                const int64_t m = acc.end() - acc.begin();
                X.ar.room(m);
                int32_t *cc = X.ar.cb.back().get() + X.ar.used;
                double *vv = X.ar.vb.back().get() + X.ar.used;
                int64_t e = 0;
                for (int32_t j : acc) {
                    cc[e] = j;
                    vv[e++] = acc.v[j];
                }
                X.ar.used += m;
                acc.clear();
                ref[i] = RowRef{cc, vv, m};
            }
        });
    }
    // the CSR (exact zeros dropped), rows in parallel
    HostCSR P;
    P.nrows = n;
    P.ncols = nc;
    P.rp.assign(n + 1, 0);
    parallel_rows(n, T, [&](int, int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            int64_t c = 0;
            for (int64_t e = 0; e < ref[i].len; ++e) c += ref[i].v[e] != 0.0;
            P.rp[i + 1] = c;
        }
    });
    for (int64_t i = 0; i < n; ++i) P.rp[i + 1] += P.rp[i];
    P.ci.resize(P.rp[n]);
    P.v.resize(P.rp[n]);
    parallel_rows(n, T, [&](int, int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            int64_t o = P.rp[i];
            for (int64_t e = 0; e < ref[i].len; ++e)
                if (ref[i].v[e] != 0.0) {
                    P.ci[o] = ref[i].c[e];
                    P.v[o++] = ref[i].v[e];
                }
        }
    });
    return P;
}

// oracle ext_i_interp()
HostCSR ext_i(const HostCSR &A, const Pattern &S, const std::vector<int8_t> &cf) {
    const int64_t n = A.nrows;
    int64_t nc = 0;
    const std::vector<int32_t> cidx = coarse_index(cf, nc);
    std::vector<double> diag(n, 0.0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k)
            if (A.ci[k] == i) diag[i] = A.v[k];
    RowSet R;
    R.col.resize(n);
    R.val.resize(n);
    const int T = setup_threads();
    // rows of very different cost (C rows are free, F rows on a dense Galerkin
    // level ~|S_i| x |A_k|): blocks of rows on demand
    struct State {
        std::vector<char> chat, strong;
        std::vector<int32_t> chat_list, fk;
        std::vector<double> fa, fD;
        Acc w;
        explicit State(int64_t n) : chat(n, 0), strong(n, 0), w(n) {}
    };
    std::vector<std::unique_ptr<State>> state(T);
    parallel_dynamic(n, T, 16, [&](int t) { state[t] = std::make_unique<State>(n); }, [&](int t, int64_t i0, int64_t i1) {
        State &X = *state[t];
        std::vector<char> &chat = X.chat, &strong = X.strong;
        std::vector<int32_t> &chat_list = X.chat_list, &fk = X.fk;
        std::vector<double> &fa = X.fa, &fD = X.fD;
        Acc &w = X.w;
        for (int64_t i = i0; i < i1; ++i) {
            if (cf[i] == CPT) {
                R.col[i] = {cidx[i]};
                R.val[i] = {1.0};
                continue;
            }
            chat_list.clear();
            for (int64_t q = S.rp[i]; q < S.rp[i + 1]; ++q) {
                const int32_t k = S.ci[q];
                strong[k] = 1;
                if (cf[k] == CPT) {
                    if (!chat[k]) chat_list.push_back(k);
                    chat[k] = 1;
                } else {
                    for (int64_t r = S.rp[k]; r < S.rp[k + 1]; ++r) {
                        const int32_t l = S.ci[r];
                        if (cf[l] == CPT && !chat[l]) {
                            chat[l] = 1;
                            chat_list.push_back(l);
                        }
                    }
                }
            }
            // every l in C^_i is entered in w up front (adding +0.0 to its +0.0), so
            // the loops below add to w.v directly
            for (int32_t l : chat_list) w.add(l, 0.0);
            double dt = 0.0;
            for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                const int32_t j = A.ci[k];
                const double a = A.v[k];
                if (j == i) dt += a;
                else if (chat[j]) w.v[j] += a;
                else if (strong[j]) continue;
                else dt += a;
            }
            // the strong F neighbours k (S_i order) with a_ik (A's row i is sorted, S_i ascending: merge)
            fk.clear();
            fa.clear();
            int64_t ak = A.rp[i];
            for (int64_t q = S.rp[i]; q < S.rp[i + 1]; ++q) {
                const int32_t k = S.ci[q];
                if (cf[k] != FPT) continue;
                while (A.ci[ak] < k) ++ak;
                fk.push_back(k);
                fa.push_back(A.v[ak]);
            }
            // D_k = sum over k's row (storage order) of a_kl with a_kl a_kk < 0 and l in C^_i or
            // l = i -- four neighbours' sums interleaved (four independent add chains; a
            // skipped entry adds +0.0, which leaves D unchanged since D is never -0.0)
            const size_t nfk = fk.size();
            fD.resize(nfk);
            chat[i] = 1;  // (the l = i case; chat holds C points only, i is F)
            for (size_t g = 0; g < nfk; g += 4) {
                int64_t b[4], len[4];
                double dk[4], D[4] = {0.0, 0.0, 0.0, 0.0};
                int64_t L = 0;
                for (int u = 0; u < 4; ++u) {
                    if (g + u < nfk) {
                        b[u] = A.rp[fk[g + u]];
                        len[u] = A.rp[fk[g + u] + 1] - b[u];
                        dk[u] = diag[fk[g + u]];
                    } else {
                        b[u] = 0;
                        len[u] = 0;
                        dk[u] = 0.0;
                    }
                    L = std::max(L, len[u]);
                }
                for (int64_t r = 0; r < L; ++r)
                    for (int u = 0; u < 4; ++u)
                        if (r < len[u]) {
                            const int64_t x = b[u] + r;
                            const double a = A.v[x];
                            D[u] += (chat[A.ci[x]] && a * dk[u] < 0.0) ? a : 0.0;
                        }
                for (int u = 0; u < 4 && g + u < nfk; ++u) fD[g + u] = D[u];
            }
            chat[i] = 0;
            for (size_t f = 0; f < nfk; ++f) {
                const int32_t k = fk[f];
                const double a_ik = fa[f];
                const double dk = diag[k];
                const double D = fD[f];
                if (D == 0.0) {
                    dt += a_ik;
                    continue;
                }
                const double distribute = a_ik / D;  // (hypre's ext+i: one division per strong F neighbour)
                // branch-free: entries outside C^_i or of the wrong sign add +0.0 to a +0.0
                // (l not in C^_i) or to a nonzero / +0.0 sum (w.v is never -0.0), i.e. nothing
                const int64_t rb = A.rp[k], re = A.rp[k + 1];
                double *wv = w.v.data();
                for (int64_t r = rb; r < re; ++r) {
                    const int32_t l = A.ci[r];
                    const double a = A.v[r];
                    wv[l] += (chat[l] && a * dk < 0.0) ? distribute * a : 0.0;
                }
                const int32_t *pi = std::lower_bound(A.ci.data() + rb, A.ci.data() + re, (int32_t)i);
                if (pi != A.ci.data() + re && *pi == i) {
                    const double a = A.v[pi - A.ci.data()];
                    if (a * dk < 0.0) dt += distribute * a;
                }
            }
            w.sort();
            if (dt != 0.0)
                for (int32_t j : w) {
                    R.col[i].push_back(cidx[j]);
                    R.val[i].push_back(-w.v[j] / dt);
                }
            w.clear();
            for (int32_t l : chat_list) chat[l] = 0;
            for (int64_t q = S.rp[i]; q < S.rp[i + 1]; ++q) strong[S.ci[q]] = 0;
        }
    });
    return to_csr(R, nc);
}

// oracle truncate(): keep the pmax largest |P_ij| (ties: smaller j), rescale
HostCSR truncate(const HostCSR &P, int64_t pmax) {
    if (pmax <= 0) return P;
    RowSet R;
    R.col.resize(P.nrows);
    R.val.resize(P.nrows);
    parallel_rows(P.nrows, setup_threads(), [&](int, int64_t i0, int64_t i1) {
        std::vector<int64_t> idx;
        for (int64_t i = i0; i < i1; ++i) {
            const int64_t b = P.rp[i], e = P.rp[i + 1];
            if (e - b <= pmax) {
                R.col[i].assign(P.ci.begin() + b, P.ci.begin() + e);
                R.val[i].assign(P.v.begin() + b, P.v.begin() + e);
                continue;
            }
            idx.resize(e - b);
            for (int64_t k = b; k < e; ++k) idx[k - b] = k;
            std::sort(idx.begin(), idx.end(), [&](int64_t x, int64_t y) {
                const double ax = std::fabs(P.v[x]), ay = std::fabs(P.v[y]);
                return ax != ay ? ax > ay : P.ci[x] < P.ci[y];
            });
            idx.resize(pmax);
            std::sort(idx.begin(), idx.end());
            double tot = 0.0, kept = 0.0;
            for (int64_t k = b; k < e; ++k) tot += P.v[k];
            for (int64_t k : idx) kept += P.v[k];
            const double s = kept != 0.0 ? tot / kept : 1.0;
            for (int64_t k : idx) {
                R.col[i].push_back(P.ci[k]);
                R.val[i].push_back(P.v[k] * s);
            }
        }
    });
    return to_csr(R, P.ncols);
}

// hypre's OpenMP partition of a level's n rows over its K_l threads (par_relax.c
// relax type 6): chunk size n / K_l, the first n % K_l chunks one row longer;
// K_l = K, fewer when a chunk would hold fewer than min_rows rows (0: no floor)
int64_t level_chunks(int64_t n, int64_t K, int64_t min_rows) {
    if (min_rows > 0) K = std::min<int64_t>(K, std::max<int64_t>(1, n / min_rows));
    return std::max<int64_t>(1, std::min<int64_t>(K, n));
}
struct ChunkMap {
    int64_t q = 1, r = 0;
    ChunkMap(int64_t n, int64_t K) : q(n / K), r(n % K) {}
    int64_t operator()(int64_t i) const { return i < r * (q + 1) ? i / (q + 1) : r + (i - r * (q + 1)) / q; }
};

// The chunk-block-diagonal part of A (entries whose row and column share a
// chunk of the level's K_l chunks) restricted to rows / columns `idx` (idx
// ascending; empty: all): part 0 all of it, 1 its lower triangle with the
// diagonal (D + L), 2 the upper one (D + U).  A zero or missing diagonal entry
// is refused (hypre would skip the row).
HostCSR chunk_part(const HostCSR &A, const std::vector<int32_t> &idx, const std::vector<int64_t> &cst, int part) {
    const int64_t n = A.nrows;
    std::vector<int32_t> cid(n);
    for (size_t k = 0; k + 1 < cst.size(); ++k)
        for (int64_t i = cst[k]; i < cst[k + 1]; ++i) cid[i] = (int32_t)k;
    std::vector<int32_t> loc;
    const bool all = idx.empty();
    if (!all) {
        loc.assign(n, -1);
        for (size_t t = 0; t < idx.size(); ++t) loc[idx[t]] = (int32_t)t;
    }
    const int64_t m = all ? n : (int64_t)idx.size();
    HostCSR T;
    T.nrows = T.ncols = m;
    T.rp.assign(m + 1, 0);
    // rows in parallel: count, then fill (the same entries in the same order)
    std::vector<int64_t> bad(setup_threads(), -1);
    auto scan = [&](int64_t r, auto emit) {
        const int64_t i = all ? r : idx[r];
        const int32_t ch = cid[i];
        bool has_diag = false;
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
            const int32_t j = all ? A.ci[k] : loc[A.ci[k]];
            if (j < 0 || (part == 1 && j > r) || (part == 2 && j < r) || cid[A.ci[k]] != ch) continue;
            if (j == r) {
                if (A.v[k] == 0.0) break;
                has_diag = true;
            }
            emit(j, A.v[k]);
        }
        return has_diag;
    };
    parallel_rows(m, setup_threads(), [&](int t, int64_t r0, int64_t r1) {
        for (int64_t r = r0; r < r1; ++r) {
            int64_t c = 0;
            if (!scan(r, [&](int32_t, double) { ++c; }) && bad[t] < 0) bad[t] = all ? r : idx[r];
            T.rp[r + 1] = c;
        }
    });
    for (int64_t b : bad)
        if (b >= 0) throw Error("boomeramg: zero diagonal entry on a Gauss-Seidel level (row " + std::to_string(b) + ")");
    for (int64_t r = 0; r < m; ++r) T.rp[r + 1] += T.rp[r];
    T.ci.resize(T.rp[m]);
    T.v.resize(T.rp[m]);
    parallel_rows(m, setup_threads(), [&](int, int64_t r0, int64_t r1) {
        for (int64_t r = r0; r < r1; ++r) {
            int64_t o = T.rp[r];
            scan(r, [&](int32_t j, double v) {
                T.ci[o] = j;
                T.v[o++] = v;
            });
        }
    });
    return T;
}

struct BParams {
    double theta = 0.25, mu = 0.9, rap_bytes = 16e9;
    int64_t pmax = 0, agg_nl = 0, max_levels = 25;
    int64_t chunks = 256, chunk_rows = 1024;  // hybrid Gauss-Seidel partition (pls.hypre_relax_*)
    int64_t coarsen_chunks = 1, coarsen_rows = 65536;  // HMIS partitions (pls.hypre_coarsen_*): 1 = none (np = 1, default), 0 = auto
    int paths = 1, K = 1;
    bool no_cf = false;
    std::string ranks;  // pls.hypre_ranks: the level-0 rank partition ("G" or "n0,n1,..."), hypre under mpirun -np G
};

// level-0 rank sizes of pls.hypre_ranks (empty: one rank)
std::vector<int64_t> rank_sizes(const std::string &spec, int64_t n) {
    std::vector<int64_t> out;
    if (spec.empty()) return out;
    if (spec.find(',') == std::string::npos) {
        const int64_t G = std::stoll(spec);
        if (G <= 1) return out;
        for (int64_t q = 0; q < G; ++q) out.push_back(n / G + (q < n % G ? 1 : 0));
        return out;
    }
    int64_t tot = 0;
    size_t a = 0;
    while (a <= spec.size()) {
        const size_t b = spec.find(',', a);
        out.push_back(std::stoll(spec.substr(a, b == std::string::npos ? std::string::npos : b - a)));
        tot += out.back();
        if (b == std::string::npos) break;
        a = b + 1;
    }
    if (tot != n) throw Error("pls.hypre_ranks: the rank sizes do not add up to the block's rows");
    return out;
}

// starts of the level's parts (sizes; zero-sized parts kept)
std::vector<int64_t> part_starts(const std::vector<int64_t> &sizes) {
    std::vector<int64_t> st(1, 0);
    for (int64_t v : sizes) st.push_back(st.back() + v);
    return st;
}

BParams parse_params(const Options &o, const std::string &prefix) {
    const std::string pre = prefix + "pc_hypre_boomeramg_";
    BParams p;
    p.theta = o.num(pre + "strong_threshold", 0.25);
    p.mu = o.num(pre + "max_row_sum", 0.9);
    p.pmax = o.integer(pre + "P_max", 0);
    p.agg_nl = o.integer(pre + "agg_nl", 0);
    p.paths = (int)o.integer(pre + "agg_num_paths", 1);
    p.max_levels = o.integer(pre + "max_levels", 25);
    p.K = (int)o.integer(pre + "grid_sweeps_all", 1);
    p.no_cf = o.flag(pre + "no_CF", false);
    p.rap_bytes = o.num("pls.amg_rap_dense_gb", 16.0) * 1e9;
    p.chunks = o.integer("pls.hypre_relax_chunks", 256);
    p.chunk_rows = o.integer("pls.hypre_relax_min_rows", 1024);
    p.coarsen_chunks = o.integer("pls.hypre_coarsen_chunks", 1);
    p.coarsen_rows = o.integer("pls.hypre_coarsen_min_rows", 65536);
    p.ranks = o.str("pls.hypre_ranks", "");
    if (p.chunks < 1 || p.chunk_rows < 0)
        throw Error("pls.hypre_relax_chunks must be >= 1 and pls.hypre_relax_min_rows >= 0");
    const std::string ct = o.str(pre + "coarsen_type", "HMIS"), it = o.str(pre + "interp_type", "ext+i");
    if (ct != "HMIS") throw Error(pre + "coarsen_type " + ct + ": only HMIS is implemented");
    if (it != "ext+i") throw Error(pre + "interp_type " + it + ": only ext+i is implemented");
    const std::string rt = o.str(pre + "relax_type_all", "symmetric-SOR/Jacobi");
    if (rt != "symmetric-SOR/Jacobi") throw Error(pre + "relax_type_all " + rt + ": only symmetric-SOR/Jacobi is implemented");
    if (p.K < 1) throw Error(pre + "grid_sweeps_all must be >= 1");
    if (p.paths < 1) throw Error(pre + "agg_num_paths must be >= 1");
    return p;
}

// The host setup (oracle PCBoomerAMG.__init__): on_level(A, cf, P, R, nc) for
// every level, then the coarsest operator is returned.  tm: stage seconds.
// a level's big host arrays are released on a detached thread (unmapping a
// few GB costs ~0.1 s per GB on the setup's critical path)
template <class T>
void free_later(T &&x) {
    std::thread([y = std::move(x)] {}).detach();
}

template <class F>
HostCSR host_setup(HostCSR A, const BParams &p, F on_level, double *tm) {
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    int64_t nlev = 0;
    // ranks (hypre under mpirun -np G): the HMIS first pass inside every rank, a
    // coarse level's rank owns the C points of its rows
    std::vector<int64_t> parts = rank_sizes(p.ranks, A.nrows);
    while (A.nrows > 9 && nlev < p.max_levels - 1) {
        double t0 = now();
        Pattern S = strength(A, p.theta, p.mu);
        tm[1] += now() - t0;
        t0 = now();
        const bool aggressive = nlev < p.agg_nl;
        std::vector<int64_t> pst;
        if (!parts.empty()) {
            pst = part_starts(parts);
        } else {
            int64_t Kc = p.coarsen_chunks == 1 ? 1
                         : p.coarsen_chunks > 1 ? p.coarsen_chunks
                                                : coarsen_partitions(S, level_chunks(A.nrows, p.chunks, p.coarsen_rows));
            Kc = std::max<int64_t>(1, std::min<int64_t>(Kc, A.nrows));
            pst = chunk_starts(A.nrows, Kc);
        }
        const std::vector<int8_t> cf = coarsen(S, aggressive, p.paths, pst);
        tm[2] += now() - t0;
        int64_t nc = 0;
        for (int8_t v : cf) nc += v == CPT;
        if (nc == 0 || nc == A.nrows) break;
        t0 = now();
        HostCSR P = aggressive ? multipass(A, S, cf) : truncate(ext_i(A, S, cf), p.pmax);
        const double tp = now();
        HostCSR R = amgh::transpose(P);
        tm[3] += now() - t0;
        if (std::getenv("PLS_AMG_TRACE"))
            fprintf(stderr, "[boomeramg level %lld] interp %.2f s, transpose %.2f s\n", (long long)nlev, tp - t0, now() - tp);
        t0 = now();
        HostCSR Ac;
        if (!galerkin_fused(A, P, nc, p.rap_bytes, Ac)) Ac = spgemm(R, spgemm(A, P));
        tm[4] += now() - t0;
        if (std::getenv("PLS_AMG_TRACE"))
            fprintf(stderr, "[boomeramg level %lld] n %lld nnz %lld -> nc %lld (P nnz %lld, Ac nnz %lld): RAP %.2f s\n",
                    (long long)nlev, (long long)A.nrows, (long long)A.ci.size(), (long long)nc, (long long)P.ci.size(),
                    (long long)Ac.ci.size(), now() - t0);
        on_level(A, cf, P, R, nc, parts);
        if (!parts.empty()) {  // the coarse level's rank sizes: C points per rank
            std::vector<int64_t> np(parts.size(), 0);
            for (size_t q = 0; q < parts.size(); ++q)
                for (int64_t i = pst[q]; i < pst[q + 1]; ++i) np[q] += cf[i] == CPT;
            parts.swap(np);
        }
        free_later(std::move(S));
        free_later(std::move(P));
        free_later(std::move(R));
        free_later(std::move(A));
        A = std::move(Ac);
        ++nlev;
    }
    return A;
}

// level count of a triangular solve with T (lower: forward, else backward);
// T couples rows only inside the chunks [cp[q], cp[q + 1]), swept in parallel
int64_t tri_levels(const HostCSR &T, bool upper, const std::vector<int64_t> &cp) {
    std::vector<int64_t> lev(T.nrows, 0);
    const int64_t nch = (int64_t)cp.size() - 1;
    std::vector<int64_t> top(setup_threads(), 0);
    parallel_rows(nch, setup_threads(), [&](int th, int64_t q0, int64_t q1) {
        for (int64_t q = q0; q < q1; ++q) {
            const int64_t a = cp[q], b = cp[q + 1];
            for (int64_t t = a; t < b; ++t) {
                const int64_t i = upper ? b - 1 - (t - a) : t;
                int64_t l = 0;
                for (int64_t k = T.rp[i]; k < T.rp[i + 1]; ++k)
                    if (T.ci[k] != i) l = std::max(l, lev[T.ci[k]] + 1);
                lev[i] = l;
                top[th] = std::max(top[th], l + 1);
            }
        }
    });
    return *std::max_element(top.begin(), top.end());
}

// Hybrid symmetric Gauss-Seidel through dense per-chunk inverses (mostly
// sequential chunks, e.g. the ~30 % dense Galerkin operators below an
// aggressive level, where every row is a level of its own): M_c^-1 =
// (D + U)_c^-1 D_c (D + L)_c^-1 is formed once per chunk on the device (two
// Gauss-Jordan inverses, a row scaling and a GEMM), and a sweep is one
// block-diagonal GEMV (8 bytes per row per chunk column, HBM-bound).
struct PCSGSDense : PC {
    int64_t ld = 64, K = 1;
    DBuf<double> Minv;
    DBuf<int32_t> cof;
    DBuf<int64_t> cptr;
    static int64_t ld_for(const std::vector<int64_t> &cp) {
        int64_t mx = 1;
        for (size_t k = 0; k + 1 < cp.size(); ++k) mx = std::max(mx, cp[k + 1] - cp[k]);
        return (mx + 63) / 64 * 64;
    }
    // rows [c0, c0 + m) of a block-diagonal T, columns shifted to the chunk
    static HostCSR chunk_block(const HostCSR &T, int64_t c0, int64_t m) {
        HostCSR B;
        B.nrows = B.ncols = m;
        B.rp.assign(1, 0);
        for (int64_t i = c0; i < c0 + m; ++i) {
            for (int64_t k = T.rp[i]; k < T.rp[i + 1]; ++k) {
                if (T.ci[k] < c0 || T.ci[k] >= c0 + m) throw Error("boomeramg: chunk block leaves its chunk");
                B.ci.push_back(T.ci[k] - (int32_t)c0);
                B.v.push_back(T.v[k]);
            }
            B.rp.push_back((int64_t)B.ci.size());
        }
        return B;
    }
    PCSGSDense(const HostCSR &lo, const HostCSR &up, const std::vector<int64_t> &cp, Ctx &c) {
        type = "sgs";
        n = lo.nrows;
        K = (int64_t)cp.size() - 1;
        ld = ld_for(cp);
        Minv.alloc(K * ld * ld);
        DBuf<double> Li(ld * ld), Ui(ld * ld), D(64 * 64), dd(ld);
        DBuf<int32_t> fail(1);
        HIPCHK(hipMemsetAsync(fail.p, 0, sizeof(int32_t), c.st));
        std::vector<double> dh(ld, 1.0);
        for (int64_t k = 0; k < K; ++k) {
            const int64_t c0 = cp[k], m = cp[k + 1] - c0;
            DevCSR Ld, Ud;
            upload(chunk_block(lo, c0, m), Ld, c);
            upload(chunk_block(up, c0, m), Ud, c);
            for (int64_t i = 0; i < m; ++i) dh[i] = lo.v[lo.rp[c0 + i + 1] - 1];  // the diagonal closes a lower row
            HIPCHK(hipMemcpyAsync(dd.p, dh.data(), sizeof(double) * ld, hipMemcpyHostToDevice, c.st));
            launch_dense_from_csr(m, ld, Ld.rp.p, Ld.ci.p, Ld.val.p, Li.p, c.st);
            launch_dense_invert(ld, Li.p, D.p, fail.p, c.st);
            launch_dense_from_csr(m, ld, Ud.rp.p, Ud.ci.p, Ud.val.p, Ui.p, c.st);
            launch_dense_invert(ld, Ui.p, D.p, fail.p, c.st);
            launch_dense_rowscale(m, ld, dd.p, Li.p, c.st);
            launch_dense_gemm(ld, Ui.p, Li.p, Minv.p + k * ld * ld, c.st);
            HIPCHK(hipGetLastError());
            c.sync();  // Ld / Ud / dh are reused or freed
        }
        int32_t hfail = 0;
        HIPCHK(hipMemcpyAsync(&hfail, fail.p, sizeof(int32_t), hipMemcpyDeviceToHost, c.st));
        std::vector<int32_t> of(n);
        for (int64_t k = 0; k < K; ++k)
            for (int64_t i = cp[k]; i < cp[k + 1]; ++i) of[i] = (int32_t)k;
        cof.alloc(std::max<int64_t>(n, 1));
        cptr.alloc(K + 1);
        HIPCHK(hipMemcpyAsync(cof.p, of.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c.st));
        HIPCHK(hipMemcpyAsync(cptr.p, cp.data(), sizeof(int64_t) * (K + 1), hipMemcpyHostToDevice, c.st));
        c.sync();
        if (hfail) throw Error("boomeramg: zero pivot in a dense Gauss-Seidel chunk");
    }
    bool reentrant() const override { return true; }
    void apply(const double *x, double *y, Ctx &c) override {
        launch_bdense_gemv(n, ld, cof.p, cptr.p, Minv.p, x, y, c.st);
    }
};

struct RelaxSet {  // the points one Gauss-Seidel pass visits (all, C or F)
    int64_t m = 0, chunks = 1;
    bool all = true;
    DBuf<int64_t> idx;
    DevCSR sub;                // C / F sets: the chunk-block-diagonal part restricted to the set
    std::unique_ptr<PC> sgs;   // r -> M^-1 r: one hybrid symmetric GS sweep from 0
};

struct BLevel {
    const DevCSR *A = nullptr;  // level 0: the PC's matrix; else Aown
    std::unique_ptr<DevCSR> Aown;
    DevCSR P, R;
    int64_t n = 0, nc = 0;
    std::vector<std::unique_ptr<RelaxSet>> sets;  // no_CF: {all}; else {C, F}
    // sharded (PCBoomer::dist): n / nc are this rank's rows; gn the level's global
    // rows, set_global the sets' sizes over all ranks
    int64_t gn = 0;
    std::vector<int64_t> set_global;
};

struct BWork {
    std::vector<DBuf<double>> r, t, x, b, xs, rs, ts;
    DBuf<double> cx, cb;
    DBuf<double> csend, cgath, cbg, cxg;  // sharded: the coarsest level's gather
};

struct PCBoomer : PC {
    std::vector<std::unique_ptr<BLevel>> lv;
    int K = 1;
    bool no_cf = false;
    bool dist = false;             // this rank's rows of hypre's np = G hierarchy (sharded block)
    int64_t nco = 0;               // coarsest level rows (all ranks)
    int64_t nco_mine = 0, coarse_a = 0, maxc = 1;  // sharded: my coarsest rows [coarse_a, + nco_mine)
    DBuf<int64_t> coarse_src;      // global coarse row -> slot in the padded allgather
    DevCSR Cinv;
    std::unique_ptr<PC> Clu;
    std::unique_ptr<DevCSR> Cmat;
    std::map<hipStream_t, std::unique_ptr<BWork>> work;

    bool reentrant() const override { return true; }

    BWork &work_for(Ctx &c) {
        auto &w = work[c.st];
        if (!w) {
            w = std::make_unique<BWork>();
            const size_t L = lv.size();
            for (auto *v : {&w->r, &w->t, &w->x, &w->b, &w->xs, &w->rs, &w->ts}) v->resize(L);
            for (size_t l = 0; l < L; ++l) {
                const size_t m = (size_t)std::max<int64_t>(lv[l]->n, 1);
                w->r[l].alloc(m);
                w->t[l].alloc(m);
                if (l > 0) {
                    w->x[l].alloc(m);
                    w->b[l].alloc(m);
                }
                if (!no_cf) {
                    w->xs[l].alloc(m);
                    w->rs[l].alloc(m);
                    w->ts[l].alloc(m);
                }
            }
            w->cx.alloc(std::max<int64_t>(nco_mine, 1));
            w->cb.alloc(std::max<int64_t>(nco_mine, 1));
            if (dist) {
                w->csend.alloc(maxc);
                HIPCHK(hipMemsetAsync(w->csend.p, 0, sizeof(double) * maxc, c.st));
                w->cgath.alloc(maxc * c.comm->size);
                w->cbg.alloc(std::max<int64_t>(nco, 1));
                w->cxg.alloc(std::max<int64_t>(nco, 1));
            }
        }
        return *w;
    }

    // the smoother of one level: hybrid symmetric Gauss-Seidel sets (no_CF: all
    // rows; else C then F) over the chunks cst of Al's rows (bounds: explicit
    // chunk starts on the device); Adev: the level's device matrix (PCILU
    // extracts each chunk's block from it; a sharded one drops its ghost columns)
    void build_sets(BLevel &L, const HostCSR &Al, const std::vector<int8_t> &cf, const std::vector<int64_t> &cst,
                    bool bounds, const DevCSR &Adev, const Options &o, const std::string &prefix, Ctx &c) {
        const bool allow_lds = o.flag("pls.ilu_lds", true);
        const int gmem = (int)o.integer("pls.ilu_gmem", 0), ring = (int)o.integer("pls.ilu_ring", 1);
        // Gauss-Seidel chunks through dense inverses: -1 by the cost model below, 1 whenever
        // they fit (pls.amg_gs_dense_gb, chunks <= pls.lu_dense_max rows), 0 never
        const int gs_dense = (int)o.integer("pls.amg_gs_dense", -1);
        const double level_us = o.num("pls.amg_gs_level_us", 0.5);  // sweep cost per level (measured ~0.3-1 us)
        const double dense_gb = o.num("pls.amg_gs_dense_gb", 2.0);
        const int64_t wide_rows = o.integer("pls.amg_wide_rows", 256);  // rows per level above which: grid-wide sweeps
        const int wide_mode = (int)o.integer("pls.amg_wide_mode", -2);  // -2: CSR level kernels, -1: SELL level slices
        const int64_t dense_max = o.integer("pls.lu_dense_max", 32768);
        std::vector<std::vector<int32_t>> groups;
        if (no_cf) {
            groups.emplace_back();
        } else {
            groups.resize(2);
            for (int64_t i = 0; i < Al.nrows; ++i) groups[cf[i] == CPT ? 0 : 1].push_back((int32_t)i);
        }
        const int64_t Kl = (int64_t)cst.size() - 1;
        for (auto &g : groups) {
            auto rs = std::make_unique<RelaxSet>();
            rs->all = no_cf;
            rs->chunks = Kl;
            rs->m = no_cf ? Al.nrows : (int64_t)g.size();
            if (rs->m > 0) {
                if (!no_cf) {
                    std::vector<int64_t> gi(g.begin(), g.end());
                    rs->idx.alloc(gi.size());
                    HIPCHK(hipMemcpyAsync(rs->idx.p, gi.data(), sizeof(int64_t) * gi.size(), hipMemcpyHostToDevice, c.st));
                }
                const HostCSR lo = chunk_part(Al, g, cst, 1), up = chunk_part(Al, g, cst, 2);
                // the set's chunk boundaries in its own numbering (chunks without set points dropped)
                std::vector<int64_t> cp{0};
                {
                    std::vector<int32_t> cid(Al.nrows);
                    for (size_t k = 0; k + 1 < cst.size(); ++k)
                        for (int64_t i = cst[k]; i < cst[k + 1]; ++i) cid[i] = (int32_t)k;
                    for (int64_t t = 1; t < rs->m; ++t)
                        if (cid[no_cf ? t : g[t]] != cid[no_cf ? t - 1 : g[t - 1]]) cp.push_back(t);
                    cp.push_back(rs->m);
                }
                // a sweep's critical path (levels of both triangles, one chunk per
                // workgroup) against the bytes of the dense chunk inverses: mostly
                // sequential chunks (every row a level of its own) go dense
                const int64_t nlev = tri_levels(lo, false, cp), nlev_u = tri_levels(up, true, cp);
                const int64_t ldc = PCSGSDense::ld_for(cp);
                const double dense_bytes = (double)((int64_t)cp.size() - 1) * ldc * ldc * 8.0;
                const double t_dense = (double)rs->m * ldc * 8.0 / 5e12 + 5e-6;
                const double t_sweep = (double)(nlev + nlev_u) * level_us * 1e-6;
                const bool dense = gs_dense != 0 && ldc <= dense_max && dense_bytes <= dense_gb * 1e9 &&
                                   (gs_dense == 1 || t_dense < t_sweep);
                if (dense) {
                    rs->sgs = std::make_unique<PCSGSDense>(lo, up, cp, c);
                } else {
                    // wide levels: one grid-wide launch per level beats one workgroup
                    const int gm = (nlev > 0 && lo.nrows / nlev > wide_rows) ? wide_mode : gmem;
                    if (no_cf) {
                        // the chunks are PCILU's blocks (the same partition): one workgroup per chunk
                        auto pc = std::make_unique<PCILU>(Adev, Kl, c, false, allow_lds, 0, gm, ring, true,
                                                          bounds ? &cst : nullptr);
                        if (o.has("pls.sweep_tpb")) pc->lds_tpb = (int)o.integer("pls.sweep_tpb", 1024);
                        if (o.has("pls.sweep_rr")) pc->lds_rr = o.flag("pls.sweep_rr", false) && pc->use_lds && !pc->ring;
                        if (o.flag("pls.sweep_profile", false))
                            pc->profile_tag = prefix + "sgs L" + std::to_string(lv.size());
                        rs->sgs = std::move(pc);
                    } else {
                        upload(chunk_part(Al, g, cst, 0), rs->sub, c);
                        rs->sgs = std::make_unique<PCILU>(rs->sub, 1, c, false, allow_lds, 0, gm, ring, true);
                    }
                }
            }
            L.sets.push_back(std::move(rs));
        }
    }

    // rows [a, a + m) of T (columns unchanged)
    static HostCSR row_range(const HostCSR &T, int64_t a, int64_t m) {
        HostCSR B;
        B.nrows = m;
        B.ncols = T.ncols;
        B.rp.assign(1, 0);
        for (int64_t i = a; i < a + m; ++i) {
            B.ci.insert(B.ci.end(), T.ci.begin() + T.rp[i], T.ci.begin() + T.rp[i + 1]);
            B.v.insert(B.v.end(), T.v.begin() + T.rp[i], T.v.begin() + T.rp[i + 1]);
            B.rp.push_back((int64_t)B.ci.size());
        }
        return B;
    }
    // rows and columns [a, a + m) of T, shifted to 0 (a rank's diagonal block)
    static HostCSR diag_block(const HostCSR &T, int64_t a, int64_t m) {
        HostCSR B;
        B.nrows = B.ncols = m;
        B.rp.assign(1, 0);
        for (int64_t i = a; i < a + m; ++i) {
            for (int64_t k = T.rp[i]; k < T.rp[i + 1]; ++k)
                if (T.ci[k] >= a && T.ci[k] < a + m) {
                    B.ci.push_back(T.ci[k] - (int32_t)a);
                    B.v.push_back(T.v[k]);
                }
            B.rp.push_back((int64_t)B.ci.size());
        }
        return B;
    }

    // M: the block (one rank), or this rank's rows of a sharded block (M.halo)
    // with `global` the gathered block and rank_rows the ranks' contiguous row
    // counts: hypre under mpirun -np G -- the hierarchy of the G-rank setup
    // (identical on every rank), each rank holding and smoothing only its rows of
    // every level (A_l, P_l with halos; R_l = its coarse rows of P_l^T), Jacobi
    // across ranks through the halo values of the residual, the coarsest level
    // gathered and solved redundantly.
    PCBoomer(const DevCSR &M, const Options &o, const std::string &prefix, Ctx &c, const HostCSR *global = nullptr,
             const std::vector<int64_t> *rank_rows = nullptr) {
        type = "hypre";
        n = M.nrows;
        dist = global != nullptr;
        BParams prm = parse_params(o, prefix);
        const std::vector<int64_t> &rr = rank_rows ? *rank_rows : c.rank_rows;
        int64_t rsum = 0;
        for (int64_t v : rr) rsum += v;
        const int64_t nglob = dist ? global->nrows : M.nrows;
        if (prm.ranks.empty() && rr.size() > 1 && rsum == nglob) {  // the G ranks' partition (hypre's np = G setup)
            for (size_t q = 0; q < rr.size(); ++q) prm.ranks += (q ? "," : "") + std::to_string(rr[q]);
        }
        if (dist && (!c.comm || (int64_t)rr.size() != c.comm->size || rsum != nglob || rr[c.comm->rank] != M.nrows))
            throw Error("boomeramg (prefix " + prefix + "): the sharded block's ranks must own contiguous rows");
        K = prm.K;
        no_cf = prm.no_cf;
        if (!M.sell) build_sell(const_cast<DevCSR &>(M), c);
        const bool view = o.flag("pls.amg_view", false);
        double tm[7] = {0};
        auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
        double t0 = now();
        std::unique_ptr<DevCSR> cur;
        const int me = dist ? c.comm->rank : 0;
        std::vector<int64_t> cps_last;  // dist: the coarsest level's rank starts
        if (std::getenv("PLS_AMG_TRACE") && !dist) {
            const double td = now();
            HostCSR Hd = download(M, c);
            fprintf(stderr, "[boomeramg %s] download %.2f s (nnz %lld)\n", prefix.c_str(), now() - td, (long long)Hd.ci.size());
        }
        HostCSR Ahost = dist ? *global : download(M, c);
        const double t_dl = now() - t0;
        HostCSR A = host_setup(std::move(Ahost), prm,
                               [&](const HostCSR &Al, const std::vector<int8_t> &cf, const HostCSR &P, const HostCSR &R,
                                   int64_t nc, const std::vector<int64_t> &parts) {
            const double t1 = now();
            auto L = std::make_unique<BLevel>();
            if (!dist) {
                L->n = Al.nrows;
                L->nc = nc;
                if (lv.empty()) {
                    L->A = &M;
                } else {  // the level's Galerkin operator
                    L->Aown = std::make_unique<DevCSR>();
                    upload(Al, *L->Aown, c);
                    amg_layout(*L->Aown, c);
                    L->A = L->Aown.get();
                }
                upload(P, L->P, c);
                upload(R, L->R, c);
                amg_layout(L->P, c);
                amg_layout(L->R, c);
                std::vector<int64_t> cst;
                if (parts.empty()) {
                    cst = chunk_starts(Al.nrows, level_chunks(Al.nrows, prm.chunks, prm.chunk_rows));
                } else {
                    // each rank's rows cut into its threads' chunks (pls.hypre_relax_chunks / ranks threads per rank)
                    cst.assign(1, 0);
                    const int64_t T = std::max<int64_t>(1, prm.chunks / (int64_t)parts.size());
                    for (int64_t sz : parts) {
                        if (sz == 0) continue;
                        const std::vector<int64_t> loc = chunk_starts(sz, level_chunks(sz, T, prm.chunk_rows));
                        const int64_t base = cst.back();
                        for (size_t k = 1; k < loc.size(); ++k) cst.push_back(base + loc[k]);
                    }
                }
                build_sets(*L, Al, cf, cst, !parts.empty(), *L->A, o, prefix, c);
            } else {
                // this rank's rows of the level (parts: the level's rank sizes) and of its coarse level
                const std::vector<int64_t> pst = part_starts(parts);
                std::vector<int64_t> cnt(parts.size(), 0);
                for (size_t q = 0; q < parts.size(); ++q)
                    for (int64_t i = pst[q]; i < pst[q + 1]; ++i) cnt[q] += cf[i] == CPT;
                const std::vector<int64_t> cps = part_starts(cnt);
                const int64_t a = pst[me], m = pst[me + 1] - a, ca = cps[me], mc = cps[me + 1] - ca;
                L->n = m;
                L->nc = mc;
                L->gn = Al.nrows;
                if (lv.empty()) {
                    L->A = &M;
                } else {
                    L->Aown = std::make_unique<DevCSR>();
                    upload_dist(row_range(Al, a, m), pst, *L->Aown, c);
                    L->A = L->Aown.get();
                }
                upload_dist(row_range(P, a, m), cps, L->P, c);
                upload_dist(row_range(R, ca, mc), pst, L->R, c);
                // the C / F set sizes over all ranks (a set is visited when any rank has points in it)
                int64_t nC = 0;
                for (int8_t v : cf) nC += v == CPT;
                L->set_global = no_cf ? std::vector<int64_t>{Al.nrows} : std::vector<int64_t>{nC, Al.nrows - nC};
                const int64_t T = std::max<int64_t>(1, prm.chunks / (int64_t)parts.size());
                const std::vector<int64_t> cst = chunk_starts(m, m > 0 ? level_chunks(m, T, prm.chunk_rows) : 1);
                const std::vector<int8_t> cfm(cf.begin() + a, cf.begin() + a + m);
                if (m > 0) {
                    build_sets(*L, diag_block(Al, a, m), cfm, cst, true, *L->A, o, prefix, c);
                } else {
                    for (size_t g = 0; g < L->set_global.size(); ++g) {
                        L->sets.push_back(std::make_unique<RelaxSet>());
                        L->sets.back()->all = no_cf;
                    }
                }
                cps_last = cps;
            }
            lv.push_back(std::move(L));
            c.sync();
            tm[5] += now() - t1;
        }, tm);
        tm[0] = now() - t0 - (tm[1] + tm[2] + tm[3] + tm[4] + tm[5]);
        if (std::getenv("PLS_AMG_TRACE"))
            fprintf(stderr, "[boomeramg %s] download/copy %.2f s, untimed in the level loop %.2f s\n", prefix.c_str(), t_dl,
                    tm[0] - t_dl);
        if (!lv.empty() || dist) {  // (sharded: the coarsest operator is the gathered global one)
            cur = std::make_unique<DevCSR>();
            upload(A, *cur, c);
            amg_layout(*cur, c);
        }
        t0 = now();
        nco = A.nrows;
        nco_mine = nco;
        if (dist) {
            if (lv.empty()) cps_last = part_starts(rr);  // the block is the coarsest level (<= 9 rows, or no coarsening)
            // the coarsest level is solved redundantly: gather b_c (padded allgather), keep my rows of x_c
            const int G = c.comm->size;
            nco_mine = cps_last[me + 1] - cps_last[me];
            coarse_a = cps_last[me];
            maxc = 1;
            for (int q = 0; q < G; ++q) maxc = std::max(maxc, cps_last[q + 1] - cps_last[q]);
            std::vector<int64_t> src(std::max<int64_t>(nco, 1), 0);
            for (int q = 0; q < G; ++q)
                for (int64_t i = cps_last[q]; i < cps_last[q + 1]; ++i) src[i] = q * maxc + (i - cps_last[q]);
            coarse_src.alloc(src.size());
            HIPCHK(hipMemcpyAsync(coarse_src.p, src.data(), sizeof(int64_t) * src.size(), hipMemcpyHostToDevice, c.st));
        }
        work_for(c);
        if (nco > 0) {
            if (nco <= 1024) {
                upload(dense_inverse(A), Cinv, c);
                amg_layout(Cinv, c);
            } else {
                Cmat = std::move(cur);
                const DevCSR &Cm = Cmat ? *Cmat : M;
                // hypre's Gaussian elimination (relax type 9): the exact device LU
                // (dense inverse, band or envelope LU by size; make_lu)
                Clu = make_lu(Cm, o, c);
            }
        }
        c.sync();
        tm[6] += now() - t0;
        // the V-cycle's vectors are sized from these: check the chain before any launch
        for (size_t l = 0; l < lv.size(); ++l) {
            const BLevel &L = *lv[l];
            const int64_t next = l + 1 < lv.size() ? lv[l + 1]->n : nco_mine;
            const bool cols_ok = dist ? true : (L.P.ncols == L.nc && L.R.ncols == L.n);
            if (L.A->nrows != L.n || L.P.nrows != L.n || !cols_ok || L.R.nrows != L.nc || next != L.nc)
                throw Error("boomeramg: inconsistent hierarchy at level " + std::to_string(l));
            for (const auto &s : L.sets)
                if (s->m > 0 && (!s->sgs || s->sgs->n != s->m)) throw Error("boomeramg: smoother size mismatch");
        }
        if (view) {
            fprintf(stderr, "[boomeramg %s] levels %zu%s:", prefix.c_str(), lv.size() + 1, dist ? " (this rank's rows)" : "");
            for (auto &L : lv)
                fprintf(stderr, " %lld(P nnz %lld, %lld GS chunks)", (long long)L->n, (long long)L->P.nnz,
                        (long long)(L->sets.empty() ? 0 : L->sets[0]->chunks));
            fprintf(stderr, " coarse %lld\n", (long long)nco);
            fprintf(stderr,
                    "[boomeramg %s] setup s: download/other %.2f strength %.2f coarsen %.2f interp %.2f RAP %.2f "
                    "smoothers+upload %.2f coarse %.2f (%d threads)\n",
                    prefix.c_str(), tm[0], tm[1], tm[2], tm[3], tm[4], tm[5], tm[6], setup_threads());
        }
    }

    // y = alpha M x + beta z on a level matrix; a sharded one with no local rows
    // still takes part in the halo exchange (the exchange is collective)
    void lspmv(const DevCSR &Mx, const double *x, double *y, Ctx &c, double alpha = 1.0, double beta = 0.0,
               const double *z = nullptr) {
        if (Mx.halo && Mx.nrows == 0) {
            Halo &H = *Mx.halo;
            launch_pack(H.nsend, H.send_idx.p, x, H.sendbuf.p, c.st);
            c.comm->exchange_dev(H.sendbuf.p, H.scnt, H.soff, H.ghost.p, H.rcnt, H.roff, c.st);
            return;
        }
        spmv(Mx, x, y, c, alpha, beta, z);
    }

    // one hybrid symmetric Gauss-Seidel sweep over set s (oracle _relax):
    // x_I += M^-1 (b - A x)_I  (x_zero: x == 0 on entry, so the residual is b)
    void sweep(BLevel &L, size_t l, RelaxSet &s, BWork &W, const double *b, double *x, bool x_zero, Ctx &c) {
        const double *r = b;
        if (!x_zero) {
            lspmv(*L.A, x, W.r[l].p, c, -1.0, 1.0, b);
            r = W.r[l].p;
        }
        if (s.m == 0) return;  // (sharded: no points of this set on this rank)
        if (s.all) {
            if (x_zero) {
                s.sgs->apply(r, x, c);
            } else {
                s.sgs->apply(r, W.t[l].p, c);
                launch_axpby(L.n, 1.0, W.t[l].p, 1.0, x, c.st);
            }
            return;
        }
        launch_gather(s.m, s.idx.p, r, W.rs[l].p, c.st);
        s.sgs->apply(W.rs[l].p, W.ts[l].p, c);
        launch_gather(s.m, s.idx.p, x, W.xs[l].p, c.st);
        launch_axpby(s.m, 1.0, W.ts[l].p, 1.0, W.xs[l].p, c.st);
        launch_scatter(s.m, s.idx.p, W.xs[l].p, x, c.st);
    }

    // grid_sweeps_all hybrid symmetric GS sweeps; down: C then F, up: F then C
    void relax(size_t l, BWork &W, const double *b, double *x, bool down, bool x_zero, Ctx &c) {
        BLevel &L = *lv[l];
        if (x_zero && !no_cf) launch_set(L.n, 0.0, x, c.st);
        for (int k = 0; k < K; ++k)
            for (size_t g = 0; g < L.sets.size(); ++g) {
                const size_t gi = down ? g : L.sets.size() - 1 - g;
                RelaxSet &s = *L.sets[gi];
                if ((dist ? L.set_global[gi] : s.m) == 0) continue;
                sweep(L, l, s, W, b, x, x_zero, c);
                x_zero = false;
            }
    }

    void coarse_solve(const double *b, double *x, Ctx &c) {
        if (nco == 0) return;
        if (Clu) Clu->apply(b, x, c);
        else spmv(Cinv, b, x, c);
    }
    // sharded: my rows of b_c -> the whole coarse b (allgather), solved redundantly, my rows of x_c kept
    void coarse_solve_dist(const double *b, double *x, BWork &W, Ctx &c) {
        if (nco == 0) return;
        if (nco_mine) launch_copy(nco_mine, b, W.csend.p, c.st);
        c.comm->allgather_dev(W.csend.p, (int)maxc, W.cgath.p, c.st);
        launch_gather(nco, coarse_src.p, W.cgath.p, W.cbg.p, c.st);
        coarse_solve(W.cbg.p, W.cxg.p, c);
        if (nco_mine) launch_copy(nco_mine, W.cxg.p + coarse_a, x, c.st);
    }

    void vcycle(size_t l, BWork &W, const double *b, double *x, Ctx &c) {
        if (l == lv.size()) {
            if (dist) coarse_solve_dist(b, x, W, c);
            else coarse_solve(b, x, c);
            return;
        }
        BLevel &L = *lv[l];
        const bool last = (l + 1 == lv.size());
        double *bc = last ? W.cb.p : W.b[l + 1].p;
        double *xc = last ? W.cx.p : W.x[l + 1].p;
        relax(l, W, b, x, true, true, c);
        lspmv(*L.A, x, W.r[l].p, c, -1.0, 1.0, b);
        lspmv(L.R, W.r[l].p, bc, c);
        vcycle(l + 1, W, bc, xc, c);
        lspmv(L.P, xc, x, c, 1.0, 1.0, x);
        relax(l, W, b, x, false, false, c);
    }

    void apply(const double *x, double *y, Ctx &c) override {
        if (n == 0 && !dist) return;
        if (lv.empty()) {
            if (dist) coarse_solve_dist(x, y, work_for(c), c);
            else coarse_solve(x, y, c);
            return;
        }
        vcycle(0, work_for(c), x, y, c);
    }
};

}  // namespace

// hypre on a sharded block (BoomerAMG under mpirun -np G): the gathered block
// sets up hypre's np = G hierarchy on every rank, each rank keeps its rows
std::unique_ptr<PC> make_boomeramg_dist(const DevCSR &M, const HostCSR &global, const std::vector<int64_t> &rank_rows,
                                        const Options &o, const std::string &prefix, Ctx &c) {
    return std::make_unique<PCBoomer>(M, o, prefix, c, &global, &rank_rows);
}

std::unique_ptr<PC> make_boomeramg(const DevCSR &M, const Options &o, const std::string &prefix, Ctx &c) {
    if (M.halo) throw Error("PC type hypre (prefix " + prefix + "): a sharded block reaches the AMG through PCRedundant");
    return std::make_unique<PCBoomer>(M, o, prefix, c);
}

// Host-only hierarchy query for the CPU tests (pls_boomeramg_host_level):
// level `level`'s n, nc, C/F marker and P (CSR) of the setup on the host matrix.
void boomeramg_host_level(const HostCSR &A, const Options &o, const std::string &prefix, int64_t level,
                          int64_t &nlevels, int64_t &n, int64_t &nc, std::vector<int8_t> &cf, HostCSR &P) {
    const BParams prm = parse_params(o, prefix);
    double tm[7] = {0};
    int64_t l = 0;
    n = nc = 0;
    HostCSR coarse = host_setup(A, prm, [&](const HostCSR &Al, const std::vector<int8_t> &cfl, const HostCSR &Pl,
                                            const HostCSR &, int64_t ncl, const std::vector<int64_t> &) {
        if (l == level) {
            n = Al.nrows;
            nc = ncl;
            cf = cfl;
            P = Pl;
        }
        ++l;
    }, tm);
    nlevels = l + 1;
    if (o.flag("pls.amg_view", false))
        fprintf(stderr, "[boomeramg host] strength %.2f coarsen %.2f interp %.2f RAP %.2f s (%d threads)\n", tm[1], tm[2],
                tm[3], tm[4], setup_threads());
    if (level == l) {  // the coarsest operator (P empty)
        n = coarse.nrows;
        P = coarse;
    }
}

}  // namespace pls
