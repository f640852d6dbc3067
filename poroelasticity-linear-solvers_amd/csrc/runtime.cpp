// runtime.cpp -- device memory, options, timers, operators, preconditioners
// and PETSc-semantics Krylov solvers of libpls.so.
//
// The Krylov algorithms follow PETSc as the reference configures it
// (reference lib/Solver.py:91-102 for the outer solver, lib/Preconditioner.py:
// 94-118 for the inner ones): GMRES with classical Gram-Schmidt, Givens
// rotations, happy-breakdown test and BuildSoln (gmres.c); CG (cg.c);
// PREONLY; KSPConvergedDefault (iterativ.c).  The scalar recurrences run on the
// host in double precision without FMA contraction (-ffp-contract=off), exactly
// as the CPU oracle evaluates them.
#include "runtime.hpp"

#include "amg_host.hpp"

#include <climits>
#include <sys/mman.h>

#include <algorithm>
#include <thread>
#include <functional>
#include <numeric>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstring>
#include <sstream>

namespace pls {

void *huge_alloc(size_t bytes) {
    const size_t len = (bytes + HUGE_ALLOC_MIN - 1) & ~(HUGE_ALLOC_MIN - 1);
    void *p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) throw std::bad_alloc();
    (void)madvise(p, len, MADV_HUGEPAGE);
    return p;
}
void huge_free(void *p, size_t bytes) {
    if (p) (void)munmap(p, (bytes + HUGE_ALLOC_MIN - 1) & ~(HUGE_ALLOC_MIN - 1));
}

// ============================================================== context ===
static CommSelf g_self_comm;

Ctx::Ctx() {
    comm = &g_self_comm;
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    partial.alloc(4096 * 136);
    partial_n = 4096 * 136;
    dscal.alloc(4096);
    HIPCHK(hipHostMalloc((void **)&hscal, sizeof(double) * 4096, hipHostMallocDefault));
    hscal_n = 4096;
}
static constexpr double CANARY_VALUE = -1.2345678901234567e300;

static void alloc_partial(Ctx &c, int64_t count) {
    c.partial.alloc(count + (c.debug_bounds ? Ctx::CANARY : 0));
    c.partial_n = count;
    if (c.debug_bounds) launch_set(Ctx::CANARY, CANARY_VALUE, c.partial.p + count, c.st);
}
void Ctx::set_debug(bool bounds, int64_t cap, bool no_grow, bool unguarded) {
    HIPCHK(hipStreamSynchronize(st));
    debug_bounds = bounds;
    debug_no_grow = no_grow;
    debug_unguarded = unguarded;
    alloc_partial(*this, cap > 0 ? cap : partial_n);
    HIPCHK(hipStreamSynchronize(st));
}
void Ctx::check_bounds() {
    if (!debug_bounds) return;
    std::vector<double> h(CANARY);
    HIPCHK(hipMemcpyAsync(h.data(), partial.p + partial_n, sizeof(double) * CANARY, hipMemcpyDeviceToHost, st));
    sync();
    for (int64_t i = 0; i < CANARY; ++i)
        if (h[i] != CANARY_VALUE)
            throw Error("pls.debug_bounds: the canary behind the reduction partials was overwritten at +" +
                        std::to_string(i) + " (room " + std::to_string(partial_n) + " doubles)");
}
double *Ctx::partials(int64_t n, int64_t cols) {
    const int64_t need = (int64_t)reduce_blocks(n) * std::max<int64_t>(cols, 1);
    if (need > partial_n && !debug_unguarded)
        throw Error("reduction partials: " + std::to_string(cols) + " reductions of " + std::to_string(n) +
                    " entries need " + std::to_string(need) + " doubles, the context holds " +
                    std::to_string(partial_n) + " (missing ensure_partial)");
    return partial.p;
}
double *Ctx::host_scalars(int64_t count) {
    if (count > hscal_n)
        throw Error("host scalar mirror: " + std::to_string(count) + " doubles requested, " + std::to_string(hscal_n) +
                    " held (missing ensure_partial)");
    return hscal;
}
void Ctx::ensure_partial(int64_t n, int64_t cols) {
    const int64_t need = (int64_t)reduce_blocks(n) * std::max<int64_t>(cols, 1);
    if (need > partial_n && !debug_no_grow) {
        HIPCHK(hipStreamSynchronize(st));
        alloc_partial(*this, need);
    }
    if (cols + 2 > hscal_n) {
        HIPCHK(hipStreamSynchronize(st));
        if (hscal) (void)hipHostFree(hscal);
        HIPCHK(hipHostMalloc((void **)&hscal, sizeof(double) * (cols + 2), hipHostMallocDefault));
        hscal_n = cols + 2;
    }
}
Ctx::~Ctx() {
    if (hscal) (void)hipHostFree(hscal);
    if (ev_x) (void)hipEventDestroy(ev_x);
    if (ev_halo) (void)hipEventDestroy(ev_halo);
    if (st_comm) (void)hipStreamDestroy(st_comm);
    if (st) (void)hipStreamDestroy(st);
}
void Ctx::ensure_scan(int64_t n) {
    size_t need = exclusive_scan_tmp_bytes(n);
    if (need > scan_tmp_bytes) {
        scan_tmp.alloc(need);
        scan_tmp_bytes = need;
    }
}
double Ctx::dot(int64_t n, const double *x, const double *y) {
    launch_dot(n, x, y, partials(n, 1), dscal.p, st);
    comm->global_sum_dev(dscal.p, 1, st);
    double *h = host_scalars(1);
    HIPCHK(hipMemcpyAsync(h, dscal.p, sizeof(double), hipMemcpyDeviceToHost, st));
    sync();
    return h[0];
}
double Ctx::norm2(int64_t n, const double *x) {
    launch_dot(n, x, x, partials(n, 1), dscal.p, st);
    comm->global_sum_dev(dscal.p, 1, st);
    double *h = host_scalars(1);
    HIPCHK(hipMemcpyAsync(h, dscal.p, sizeof(double), hipMemcpyDeviceToHost, st));
    sync();
    return std::sqrt(h[0]);
}

// ================================================================== CSR ===
void upload_csr(DevCSR &M, int64_t nrows, int64_t ncols, const int64_t *rp, const int32_t *ci, const double *val,
                Ctx &c) {
    M.nrows = nrows;
    M.ncols = ncols;
    M.nnz = rp[nrows] - rp[0];
    if (rp[0] != 0) throw Error("CSR row_ptr must start at 0");
    int64_t mr = 0;
    for (int64_t i = 0; i < nrows; ++i) {
        const int64_t l = rp[i + 1] - rp[i];
        if (l < 0) throw Error("CSR row_ptr not monotone");
        mr = std::max(mr, l);
        for (int64_t k = rp[i] + 1; k < rp[i + 1]; ++k)
            if (ci[k] <= ci[k - 1]) throw Error("CSR columns must be strictly ascending within a row");
        if (l > 0 && (ci[rp[i]] < 0 || ci[rp[i + 1] - 1] >= ncols)) throw Error("CSR column index out of range");
    }
    M.max_row = mr;
    M.rp.alloc(nrows + 1);
    M.ci.alloc(std::max<int64_t>(M.nnz, 1));
    M.val.alloc(std::max<int64_t>(M.nnz, 1));
    HIPCHK(hipMemcpyAsync(M.rp.p, rp, sizeof(int64_t) * (nrows + 1), hipMemcpyHostToDevice, c.st));
    if (M.nnz) {
        HIPCHK(hipMemcpyAsync(M.ci.p, ci, sizeof(int32_t) * M.nnz, hipMemcpyHostToDevice, c.st));
        HIPCHK(hipMemcpyAsync(M.val.p, val, sizeof(double) * M.nnz, hipMemcpyHostToDevice, c.st));
    }
    c.sync();
}

static int64_t max_row_of(const DBuf<int64_t> &rp, int64_t nrows, Ctx &c) {
    std::vector<int64_t> h(nrows + 1);
    HIPCHK(hipMemcpyAsync(h.data(), rp.p, sizeof(int64_t) * (nrows + 1), hipMemcpyDeviceToHost, c.st));
    c.sync();
    int64_t m = 0;
    for (int64_t i = 0; i < nrows; ++i) m = std::max(m, h[i + 1] - h[i]);
    return m;
}

void extract_csr(const DevCSR &src, int64_t r0, int64_t r1, WindowSpec w, int64_t cshift, int64_t ncols,
                 DevCSR &dst, Ctx &c) {
    const int64_t nl = r1 - r0;
    dst.sell.reset();  // re-extraction (matrix update): the SpMV layout is rebuilt on demand
    dst.halo.reset();
    DBuf<int64_t> len(nl + 1);
    launch_extract_count(src.rp.p, src.ci.p, r0, r1, w, len.p, c.st);
    dst.rp.alloc(nl + 1);
    c.ensure_scan(nl);
    exclusive_scan_i64(len.p, dst.rp.p, nl, c.scan_tmp.p, c.scan_tmp_bytes, c.st);
    int64_t nnz = 0;
    HIPCHK(hipMemcpyAsync(&nnz, dst.rp.p + nl, sizeof(int64_t), hipMemcpyDeviceToHost, c.st));
    c.sync();
    dst.nrows = nl;
    dst.ncols = ncols;
    dst.nnz = nnz;
    dst.ci.alloc(std::max<int64_t>(nnz, 1));
    dst.val.alloc(std::max<int64_t>(nnz, 1));
    launch_extract_fill(src.rp.p, src.ci.p, src.val.p, r0, r1, w, cshift, dst.rp.p, dst.ci.p, dst.val.p, c.st);
    HIPCHK(hipGetLastError());
    dst.max_row = max_row_of(dst.rp, nl, c);
}

// Slice plan of the D16 layout: per 64-row group, 8 lanes per row when the
// group's rows are "wide" (first columns of neighbouring rows more than 4
// apart on average, rows of 16+ entries: a lane-per-row gather would touch a
// cache line per lane), else lane = row.
//
// Rows of very different lengths in one slice pad every lane to the longest
// (FE systems in a bandwidth-reducing order interleave P2 vertex, P2 edge and
// P1 rows of 89..405 entries: ~100 % padding, 1.7x the CSR bytes).  When the
// padding exceeds pls.d16_sigma_pad (15 %), the plan becomes SELL-C-sigma:
// inside windows of pls.d16_sigma (1024) rows the rows are stably sorted by
// length (rowmap[position] = row; the kernel writes y[rowmap[pos]]), and each
// 64-row group of positions takes pls.d16_sorted_lpr (2) lanes per row when
// its rows average 32+ entries (keeps a gather instruction on few cache
// lines), else 1.  Per-row summation order is unchanged for lane-per-row
// slices; it is the sorted plan only if it saves 15 % of the stored entries.
static int64_t d16_plan_stored(const std::vector<int64_t> &rp, const std::vector<int64_t> &sfirst,
                               const std::vector<int32_t> &slpr, const std::vector<int32_t> *rowmap) {
    int64_t stored = 0;
    for (size_t s = 0; s + 1 < sfirst.size(); ++s) {
        const int l = slpr[s];
        int64_t L = 0;
        for (int64_t p = sfirst[s]; p < sfirst[s + 1]; ++p) {
            const int64_t r = rowmap ? (*rowmap)[p] : p;
            L = std::max<int64_t>(L, (rp[r + 1] - rp[r] + l - 1) / l);
        }
        stored += 64 * ((L + 7) & ~(int64_t)7);
    }
    return stored;
}

static void d16_plan(const DevCSR &M, std::vector<int64_t> &sfirst, std::vector<int32_t> &slpr,
                     std::vector<int32_t> &rowmap, Ctx &c, const std::vector<int32_t> *subset = nullptr) {
    const int64_t n = M.nrows;
    std::vector<int64_t> rp(n + 1);
    std::vector<int32_t> c0(n);
    DBuf<int32_t> dc0(std::max<int64_t>(n, 1));
    launch_first_col(n, M.rp.p, M.ci.p, dc0.p, c.st);
    HIPCHK(hipMemcpyAsync(rp.data(), M.rp.p, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, c.st));
    HIPCHK(hipMemcpyAsync(c0.data(), dc0.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c.st));
    c.sync();
    sfirst.clear();
    slpr.clear();
    rowmap.clear();
    if (subset) {
        // the rows left to the D16 part by the B3 layout: always the sorted plan
        std::vector<int32_t> rm(*subset);
        const int64_t m = (int64_t)rm.size();
        for (int64_t w = 0; w < m; w += std::max(c.d16_sigma, 64)) {
            const int64_t e = std::min<int64_t>(m, w + std::max(c.d16_sigma, 64));
            std::stable_sort(rm.begin() + w, rm.begin() + e,
                             [&](int32_t a, int32_t b) { return rp[a + 1] - rp[a] > rp[b + 1] - rp[b]; });
        }
        for (int64_t p = 0; p < m; p += 64) {
            const int64_t e = std::min<int64_t>(m, p + 64);
            int64_t tot = 0;
            for (int64_t q = p; q < e; ++q) tot += rp[rm[q] + 1] - rp[rm[q]];
            const int l = (c.d16_sorted_lpr > 1 && tot >= 32 * (e - p)) ? c.d16_sorted_lpr : 1;
            for (int64_t q = p; q < e; q += 64 / l) {
                sfirst.push_back(q);
                slpr.push_back(l);
            }
        }
        sfirst.push_back(m);
        rowmap.swap(rm);
        return;
    }
    for (int64_t r = 0; r < n; r += 64) {
        bool wide = false;
        if (r + 64 <= n && c0[r] >= 0 && c0[r + 63] >= 0) {
            const int64_t spread = (int64_t)c0[r + 63] - (int64_t)c0[r];
            const int64_t avg = (rp[r + 64] - rp[r]) / 64;
            wide = spread > 4 * 63 && avg >= 16;
        }
        if (wide) {
            const int l = c.d16_wide_lpr;
            for (int q = 0; q < l; ++q) {
                sfirst.push_back(r + (64 / l) * q);
                slpr.push_back(l);
            }
        } else {
            sfirst.push_back(r);
            slpr.push_back(1);
        }
    }
    sfirst.push_back(n);
    if (c.d16_sigma <= 0 || M.halo || n < 64) return;
    const int64_t nnz = rp[n];
    const int64_t stored = d16_plan_stored(rp, sfirst, slpr, nullptr);
    if ((double)stored <= (1.0 + c.d16_sigma_pad) * (double)nnz) return;
    // SELL-C-sigma
    std::vector<int32_t> rm(n);
    std::iota(rm.begin(), rm.end(), 0);
    for (int64_t w = 0; w < n; w += c.d16_sigma) {
        const int64_t e = std::min<int64_t>(n, w + c.d16_sigma);
        std::stable_sort(rm.begin() + w, rm.begin() + e, [&](int32_t a, int32_t b) {
            return rp[a + 1] - rp[a] > rp[b + 1] - rp[b];
        });
    }
    std::vector<int64_t> sf;
    std::vector<int32_t> sl;
    // entries a group of positions [p, e) stores with l lanes per row
    auto group_stored = [&](int64_t p, int64_t e, int l) {
        int64_t st = 0;
        for (int64_t q = p; q < e; q += 64 / l) {
            int64_t L = 0;
            for (int64_t t = q; t < std::min(e, q + 64 / l); ++t) L = std::max<int64_t>(L, (rp[rm[t] + 1] - rp[rm[t]] + l - 1) / l);
            st += 64 * ((L + 7) & ~(int64_t)7);
        }
        return st;
    };
    for (int64_t p = 0; p < n; p += 64) {
        const int64_t e = std::min<int64_t>(n, p + 64);
        int64_t tot = 0;
        for (int64_t q = p; q < e; ++q) tot += rp[rm[q] + 1] - rp[rm[q]];
        // several lanes per row only for long rows, and only when the per-lane
        // share's rounding to 8-entry groups costs little extra padding
        int l = 1;
        if (c.d16_sorted_lpr > 1 && tot >= 32 * (e - p) &&
            (double)group_stored(p, e, c.d16_sorted_lpr) <= 1.05 * (double)group_stored(p, e, 1))
            l = c.d16_sorted_lpr;
        for (int64_t q = p; q < e; q += 64 / l) {
            sf.push_back(q);
            sl.push_back(l);
        }
    }
    sf.push_back(n);
    const int64_t stored2 = d16_plan_stored(rp, sf, sl, &rm);
    if ((double)stored2 > 0.85 * (double)stored) return;
    sfirst.swap(sf);
    slpr.swap(sl);
    rowmap.swap(rm);
}

// SELL/B3: row triples with one column list (the components of a P2 node in
// an FE vector field).  Used when such triples hold >= half the entries; the
// other rows go to a D16 part (returned in `singles`).  Triples are sorted by
// length inside windows of 512 (SELL-C-sigma); slices of 64 / b3_lanes_per_triple() triples.
static bool build_b3(const DevCSR &M, DevSELL &S, std::vector<int32_t> &singles, Ctx &c) {
    const int64_t n = M.nrows;
    if (!c.spmv_b3 || M.halo || n < 192) return false;
    DBuf<uint8_t> df(n);
    launch_triple_flags(n, M.rp.p, M.ci.p, df.p, c.st);
    std::vector<uint8_t> f(n);
    std::vector<int64_t> rp(n + 1);
    HIPCHK(hipMemcpyAsync(f.data(), df.p, n, hipMemcpyDeviceToHost, c.st));
    HIPCHK(hipMemcpyAsync(rp.data(), M.rp.p, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, c.st));
    c.sync();
    std::vector<int32_t> heads;
    singles.clear();
    int64_t tnnz = 0;
    for (int64_t r = 0; r < n;) {
        if (f[r]) {
            heads.push_back((int32_t)r);
            tnnz += 3 * (rp[r + 1] - rp[r]);
            r += 3;
        } else {
            singles.push_back((int32_t)r);
            r += 1;
        }
    }
    if (2 * tnnz < M.nnz) return false;
    const int64_t nt = (int64_t)heads.size(), W = 512;
    for (int64_t w = 0; w < nt; w += W) {
        const int64_t e = std::min(nt, w + W);
        std::stable_sort(heads.begin() + w, heads.begin() + e,
                         [&](int32_t a, int32_t b) { return rp[a + 1] - rp[a] > rp[b + 1] - rp[b]; });
    }
    const int64_t lpt = b3_lanes_per_triple(), per = 64 / lpt, ns = (nt + per - 1) / per;
    std::vector<int64_t> bptr(ns + 1, 0);
    for (int64_t sl = 0; sl < ns; ++sl) {
        int64_t L = 0;
        for (int64_t t = sl * per; t < std::min(nt, sl * per + per); ++t)
            L = std::max<int64_t>(L, (rp[heads[t] + 1] - rp[heads[t]] + lpt - 1) / lpt);
        bptr[sl + 1] = bptr[sl] + 64 * L;
    }
    S.b3_nslices = ns;
    S.b3_ntrip = nt;
    S.b3_stored = bptr[ns];
    S.b3ptr.alloc(ns + 1);
    S.b3map.alloc(std::max<int64_t>(nt, 1));
    S.b3col.alloc(std::max<int64_t>(S.b3_stored, 1));
    S.b3val.alloc(std::max<int64_t>(3 * S.b3_stored, 1));
    HIPCHK(hipMemcpyAsync(S.b3ptr.p, bptr.data(), sizeof(int64_t) * (ns + 1), hipMemcpyHostToDevice, c.st));
    HIPCHK(hipMemcpyAsync(S.b3map.p, heads.data(), sizeof(int32_t) * nt, hipMemcpyHostToDevice, c.st));
    launch_b3_fill(ns, nt, S.b3ptr.p, S.b3map.p, M.rp.p, M.ci.p, M.val.p, S.b3col.p, S.b3val.p, c.st);
    HIPCHK(hipGetLastError());
    c.sync();
    return true;
}

// Reverse Cuthill-McKee order of a square pattern (host): per component, BFS
// from a pseudo-peripheral vertex visiting neighbours by increasing degree,
// then reversed.  order[new] = old.
static std::vector<int32_t> rcm_order(const hvec<int64_t> &rp, const hvec<int32_t> &ci, int64_t n) {
    std::vector<int32_t> order, lev(n, -1);
    order.reserve(n);
    std::vector<char> done(n, 0);
    auto deg = [&](int32_t v) { return rp[v + 1] - rp[v]; };
    std::vector<int32_t> q, nb;
    auto bfs_last = [&](int32_t s) {  // last vertex of a plain BFS (pseudo-peripheral sweep)
        q.assign(1, s);
        lev[s] = 0;
        for (size_t h = 0; h < q.size(); ++h)
            for (int64_t k = rp[q[h]]; k < rp[q[h] + 1]; ++k)
                if (lev[ci[k]] < 0 && !done[ci[k]]) {
                    lev[ci[k]] = lev[q[h]] + 1;
                    q.push_back(ci[k]);
                }
        const int32_t last = q.back();
        for (int32_t v : q) lev[v] = -1;
        return last;
    };
    for (int64_t s0 = 0; s0 < n; ++s0) {
        if (done[s0]) continue;
        int32_t s = bfs_last(bfs_last((int32_t)s0));
        size_t h = order.size();
        order.push_back(s);
        done[s] = 1;
        for (; h < order.size(); ++h) {
            const int32_t u = order[h];
            nb.clear();
            for (int64_t k = rp[u]; k < rp[u + 1]; ++k)
                if (!done[ci[k]]) {
                    done[ci[k]] = 1;
                    nb.push_back(ci[k]);
                }
            std::stable_sort(nb.begin(), nb.end(), [&](int32_t a, int32_t b) { return deg(a) < deg(b); });
            order.insert(order.end(), nb.begin(), nb.end());
        }
    }
    std::reverse(order.begin(), order.end());
    return order;
}

// The D16 layout of M with rows and columns relabelled by RCM (FE matrices:
// the caller's order interleaves P2 vertex, P2 edge and P1 dofs, so a slice's
// rows gather x from several far-apart ranges); the slices map back to M's
// rows through rowmap, and x is gathered into the RCM order before each product.
static bool build_sell_rcm(DevCSR &M, Ctx &c) {
    const int64_t n = M.nrows;
    const HostCSR H = download(M, c);
    const std::vector<int32_t> ord = rcm_order(H.rp, H.ci, n);
    std::vector<int32_t> inv(n);
    for (int64_t i = 0; i < n; ++i) inv[ord[i]] = (int32_t)i;
    HostCSR P;
    P.nrows = P.ncols = n;
    P.rp.assign(n + 1, 0);
    P.ci.resize(H.ci.size());
    P.v.resize(H.v.size());
    std::vector<std::pair<int32_t, double>> row;
    for (int64_t i = 0; i < n; ++i) {
        const int32_t o = ord[i];
        row.clear();
        for (int64_t k = H.rp[o]; k < H.rp[o + 1]; ++k) row.emplace_back(inv[H.ci[k]], H.v[k]);
        std::sort(row.begin(), row.end(), [](auto &a, auto &b) { return a.first < b.first; });
        for (size_t t = 0; t < row.size(); ++t) {
            P.ci[P.rp[i] + t] = row[t].first;
            P.v[P.rp[i] + t] = row[t].second;
        }
        P.rp[i + 1] = P.rp[i] + (int64_t)row.size();
    }
    DevCSR Mp;
    upload(P, Mp, c);
    const int keep = c.spmv_rcm;
    c.spmv_rcm = 0;
    build_sell(Mp, c);
    c.spmv_rcm = keep;
    if (!Mp.sell || !Mp.sell->d16 || Mp.sell->b3_nslices) return false;
    DevSELL &S = *Mp.sell;
    std::vector<int32_t> rm(n);
    if (S.nrows_mapped) {
        HIPCHK(hipMemcpyAsync(rm.data(), S.rowmap.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c.st));
        c.sync();
        for (auto &r : rm) r = ord[r];
    } else {
        rm = ord;
    }
    S.rowmap.alloc(n);
    S.nrows_mapped = n;
    HIPCHK(hipMemcpyAsync(S.rowmap.p, rm.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c.st));
    S.xperm.alloc(n);
    HIPCHK(hipMemcpyAsync(S.xperm.p, ord.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c.st));
    S.nperm = n;
    if (c.rcm_x.n < (size_t)n) c.rcm_x.alloc(n);
    c.sync();
    M.sell = std::move(Mp.sell);
    return true;
}

void build_sell(DevCSR &M, Ctx &c) {
    if (M.sell || M.nrows == 0) return;
    if (c.spmv_rcm != 0 && c.sell_d16 && !c.spmv_b3 && !M.halo && M.nrows == M.ncols && M.nrows >= 16384) {
        bool pads = c.spmv_rcm == 1;
        if (!pads && M.rcm_auto) {  // only where the plain plan pads (FE): the synthetic blocks keep their layout
            std::vector<int64_t> sf;
            std::vector<int32_t> lp, rm;
            d16_plan(M, sf, lp, rm, c);
            pads = !rm.empty();
        }
        if (pads && build_sell_rcm(M, c)) return;
    }
    auto S = std::make_unique<DevSELL>();
    if (c.sell_d16 && M.nnz > 0) {
        std::vector<int64_t> sf;
        std::vector<int32_t> lp, rm, singles;
        const bool b3 = build_b3(M, *S, singles, c);
        d16_plan(M, sf, lp, rm, c, b3 ? &singles : nullptr);
        const int64_t ns = (int64_t)lp.size();
        if (ns == 0) {  // every row in a triple: the B3 part is the whole product
            S->d16 = true;
            M.sell = std::move(S);
            return;
        }
        S->sfirst.alloc(ns + 1);
        S->slpr.alloc(std::max<int64_t>(ns, 1));
        HIPCHK(hipMemcpyAsync(S->sfirst.p, sf.data(), sizeof(int64_t) * (ns + 1), hipMemcpyHostToDevice, c.st));
        HIPCHK(hipMemcpyAsync(S->slpr.p, lp.data(), sizeof(int32_t) * ns, hipMemcpyHostToDevice, c.st));
        if (!rm.empty()) {
            S->rowmap.alloc(rm.size());
            S->nrows_mapped = (int64_t)rm.size();
            HIPCHK(hipMemcpyAsync(S->rowmap.p, rm.data(), sizeof(int32_t) * rm.size(), hipMemcpyHostToDevice, c.st));
        }
        const int32_t *rmap = rm.empty() ? nullptr : S->rowmap.p;
        DBuf<int32_t> mx(1);
        HIPCHK(hipMemsetAsync(mx.p, 0, sizeof(int32_t), c.st));
        launch_d16_count(ns, S->sfirst.p, S->slpr.p, M.rp.p, M.ci.p, M.nrows, mx.p, c.st, rmap);
        int32_t h = 0;
        HIPCHK(hipMemcpyAsync(&h, mx.p, sizeof(int32_t), hipMemcpyDeviceToHost, c.st));
        c.sync();
        S->d16 = h <= D16_SEG_MAX;
        S->nsegs = (h <= D16_SEG && c.d16_segs <= D16_SEG) ? D16_SEG : D16_SEG_MAX;
        if (S->d16) {
            S->nslices = ns;
            for (int32_t l : lp) S->wide_slices += (l > 1);
            DBuf<int64_t> slen(ns + 1);
            launch_d16_slice_len(ns, S->sfirst.p, S->slpr.p, M.rp.p, M.nrows, slen.p, c.st, rmap);
            S->sptr.alloc(ns + 1);
            c.ensure_scan(ns);
            exclusive_scan_i64(slen.p, S->sptr.p, ns, c.scan_tmp.p, c.scan_tmp_bytes, c.st);
            HIPCHK(hipMemcpyAsync(&S->stored, S->sptr.p + ns, sizeof(int64_t), hipMemcpyDeviceToHost, c.st));
            c.sync();
            S->val.alloc(std::max<int64_t>(S->stored, 2));
            S->dl.alloc(std::max<int64_t>(S->stored, 8));
            S->seg.alloc(ns * 64 * S->nsegs);
            launch_d16_fill(ns, S->sfirst.p, S->slpr.p, M.rp.p, M.ci.p, M.val.p, M.nrows, S->sptr.p, S->dl.p,
                            S->val.p, S->seg.p, S->nsegs, c.st, rmap);
            HIPCHK(hipGetLastError());
            c.sync();
            M.sell = std::move(S);
            if (M.halo) classify_halo_slices(M, c);
            return;
        }
        if (b3) {  // the other rows do not fit D16: plain layouts for the whole matrix
            const bool keep = c.spmv_b3;
            c.spmv_b3 = false;
            build_sell(M, c);
            c.spmv_b3 = keep;
            return;
        }
        S = std::make_unique<DevSELL>();
    }
    S->nslices = sell_nslices(M.nrows);
    DBuf<int64_t> slen(S->nslices + 1);
    launch_sell_slice_len(M.nrows, M.rp.p, slen.p, c.st);
    S->sptr.alloc(S->nslices + 1);
    c.ensure_scan(S->nslices);
    exclusive_scan_i64(slen.p, S->sptr.p, S->nslices, c.scan_tmp.p, c.scan_tmp_bytes, c.st);
    HIPCHK(hipMemcpyAsync(&S->stored, S->sptr.p + S->nslices, sizeof(int64_t), hipMemcpyDeviceToHost, c.st));
    c.sync();
    S->val.alloc(std::max<int64_t>(S->stored, 2));
    S->col.alloc(std::max<int64_t>(S->stored, 1));
    launch_sell_fill(M.nrows, M.rp.p, M.ci.p, M.val.p, S->sptr.p, S->col.p, S->val.p, c.st);
    HIPCHK(hipGetLastError());
    c.sync();
    M.sell = std::move(S);
}

void classify_halo_slices(DevCSR &M, Ctx &c) {
    if (!M.halo || !M.sell || !M.sell->d16) return;
    DevSELL &S = *M.sell;
    const int64_t n = M.nrows, ns = S.nslices;
    DBuf<uint8_t> f(std::max<int64_t>(n, 1));
    launch_row_has_ghost(n, M.rp.p, M.ci.p, M.halo->nlocal, f.p, c.st);
    std::vector<uint8_t> hf(std::max<int64_t>(n, 1));
    std::vector<int64_t> sf(ns + 1);
    if (n) HIPCHK(hipMemcpyAsync(hf.data(), f.p, n, hipMemcpyDeviceToHost, c.st));
    HIPCHK(hipMemcpyAsync(sf.data(), S.sfirst.p, sizeof(int64_t) * (ns + 1), hipMemcpyDeviceToHost, c.st));
    c.sync();
    std::vector<int32_t> in, halo;
    for (int64_t s = 0; s < ns; ++s) {
        bool g = false;
        for (int64_t r = sf[s]; r < std::min<int64_t>(sf[s + 1], n) && !g; ++r) g = hf[r] != 0;
        (g ? halo : in).push_back((int32_t)s);
    }
    S.n_in = (int64_t)in.size();
    S.n_halo = (int64_t)halo.size();
    S.s_in.alloc(std::max<int64_t>(S.n_in, 1));
    S.s_halo.alloc(std::max<int64_t>(S.n_halo, 1));
    if (S.n_in) HIPCHK(hipMemcpyAsync(S.s_in.p, in.data(), sizeof(int32_t) * S.n_in, hipMemcpyHostToDevice, c.st));
    if (S.n_halo)
        HIPCHK(hipMemcpyAsync(S.s_halo.p, halo.data(), sizeof(int32_t) * S.n_halo, hipMemcpyHostToDevice, c.st));
    c.sync();
}

void spmv(const DevCSR &M, const double *x, double *y, Ctx &c, double alpha, double beta, const double *z) {
    const double *ghost = nullptr;
    int64_t nlocal = M.ncols;
    if (M.halo && c.halo_overlap && M.sell && M.sell->d16 && M.sell->n_halo + M.sell->n_in == M.sell->nslices) {
        // interior slices on the solver stream while the pack + exchange run on
        // the comm stream; the halo slices after the exchange.  Per-row sums
        // are the kernel's as in the plain path (same result bitwise).  NCCL
        // operations never overlap: the exchange waits for everything before
        // this product on the solver stream, and the solver stream waits for
        // the exchange before the halo slices (and any later collective).
        Halo &H = *M.halo;
        const DevSELL &S = *M.sell;
        if (!c.st_comm) {
            HIPCHK(hipStreamCreateWithFlags(&c.st_comm, hipStreamNonBlocking));
            HIPCHK(hipEventCreateWithFlags(&c.ev_x, hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&c.ev_halo, hipEventDisableTiming));
        }
        HIPCHK(hipEventRecord(c.ev_x, c.st));
        HIPCHK(hipStreamWaitEvent(c.st_comm, c.ev_x, 0));
        launch_d16_spmv(M.nrows, S.n_in, S.sptr.p, S.sfirst.p, S.slpr.p, S.dl.p, S.val.p, S.seg.p, S.nsegs, x, y,
                        alpha, beta, z, M.tag, nullptr, H.nlocal, c.d16_unroll, c.st, S.s_in.p,
                        S.nrows_mapped ? S.rowmap.p : nullptr);
        launch_pack(H.nsend, H.send_idx.p, x, H.sendbuf.p, c.st_comm);
        c.comm->exchange_dev(H.sendbuf.p, H.scnt, H.soff, H.ghost.p, H.rcnt, H.roff, c.st_comm);
        HIPCHK(hipEventRecord(c.ev_halo, c.st_comm));
        HIPCHK(hipStreamWaitEvent(c.st, c.ev_halo, 0));
        launch_d16_spmv(M.nrows, S.n_halo, S.sptr.p, S.sfirst.p, S.slpr.p, S.dl.p, S.val.p, S.seg.p, S.nsegs, x, y,
                        alpha, beta, z, M.tag, H.ghost.p, H.nlocal, c.d16_unroll, c.st, S.s_halo.p,
                        S.nrows_mapped ? S.rowmap.p : nullptr);
        return;
    }
    if (M.halo) {
        Halo &H = *M.halo;
        launch_pack(H.nsend, H.send_idx.p, x, H.sendbuf.p, c.st);
        c.comm->exchange_dev(H.sendbuf.p, H.scnt, H.soff, H.ghost.p, H.rcnt, H.roff, c.st);
        ghost = H.ghost.p;
        nlocal = H.nlocal;
        if (!M.sell) throw Error("distributed matrix without SELL layout");
    }
    if (M.sell && M.sell->d16) {
        DevSELL &S = *M.sell;
        if (S.nperm) {  // RCM-relabelled columns: x in that order first (the context's scratch)
            if (c.rcm_x.n < (size_t)S.nperm) {  // a context other than the one the layout was built on
                HIPCHK(hipStreamSynchronize(c.st));
                c.rcm_x.alloc(S.nperm);
            }
            launch_gather_i32(S.nperm, S.xperm.p, x, c.rcm_x.p, c.st);
            x = c.rcm_x.p;
        }
        if (S.b3_nslices)
            launch_b3_spmv(S.b3_nslices, S.b3_ntrip, S.b3ptr.p, S.b3map.p, S.b3col.p, S.b3val.p, x, y, alpha, beta, z,
                           M.tag, c.st);
        launch_d16_spmv(M.nrows, S.nslices, S.sptr.p, S.sfirst.p, S.slpr.p, S.dl.p, S.val.p, S.seg.p, S.nsegs, x, y, alpha,
                        beta, z, M.tag, ghost, nlocal, c.d16_unroll, c.st, nullptr,
                        S.nrows_mapped ? S.rowmap.p : nullptr);
        return;
    }
    if (M.sell) {
        launch_sell_spmv(M.nrows, M.sell->sptr.p, M.sell->col.p, M.sell->val.p, x, y, alpha, beta, z, M.tag, ghost,
                         nlocal, c.st);
        return;
    }
    launch_spmv(M.nrows, M.nnz, M.rp.p, M.ci.p, M.val.p, x, y, alpha, beta, z, c.st);
}

// the slices slist[0 .. count) of a D16 layout (rows of those slices only; the
// per-row sums are spmv()'s): the 2-way PC's pressure-first pipeline
void spmv_slices(const DevCSR &M, const double *x, double *y, Ctx &c, double alpha, double beta, const double *z,
                 const int32_t *slist, int64_t count, size_t lds_reserve) {
    if (!M.sell || !M.sell->d16 || M.halo || M.sell->nperm || M.sell->b3_nslices || M.sell->nrows_mapped)
        throw Error("spmv_slices: plain D16 layouts only");
    const DevSELL &S = *M.sell;
    launch_d16_spmv(M.nrows, count, S.sptr.p, S.sfirst.p, S.slpr.p, S.dl.p, S.val.p, S.seg.p, S.nsegs, x, y, alpha, beta,
                    z, M.tag, nullptr, M.ncols, c.d16_unroll, c.st, slist, nullptr, lds_reserve);
}

// ============================================================== options ===
void Options::parse(const char *text) {
    if (!text) return;
    std::istringstream is(text);
    std::string line;
    while (std::getline(is, line)) {
        // trim
        size_t a = line.find_first_not_of(" \t\r");
        if (a == std::string::npos) continue;
        size_t b = line.find_last_not_of(" \t\r");
        line = line.substr(a, b - a + 1);
        size_t sp = line.find(' ');
        std::string k = line.substr(0, sp), v;
        if (sp != std::string::npos) {
            size_t vs = line.find_last_of(' ');
            v = line.substr(vs + 1);
        }
        while (!k.empty() && k[0] == '-') k.erase(0, 1);
        kv[k] = v;
    }
}
std::string Options::str(const std::string &k, const std::string &d) const {
    auto it = kv.find(k);
    return it == kv.end() || it->second.empty() ? d : it->second;
}
double Options::num(const std::string &k, double d) const {
    auto it = kv.find(k);
    if (it == kv.end() || it->second.empty()) return d;
    try { return std::stod(it->second); } catch (...) { throw Error("option " + k + ": not a number: " + it->second); }
}
int64_t Options::integer(const std::string &k, int64_t d) const {
    auto it = kv.find(k);
    if (it == kv.end() || it->second.empty()) return d;
    try { return (int64_t)std::stoll(it->second); } catch (...) { throw Error("option " + k + ": not an integer: " + it->second); }
}
bool Options::flag(const std::string &k, bool d) const {
    auto it = kv.find(k);
    if (it == kv.end()) return d;
    const std::string &v = it->second;
    if (v.empty() || v == "1" || v == "true" || v == "yes" || v == "on" || v == "True" || v == "TRUE") return true;
    return false;
}

// =============================================================== timers ===
Timers::~Timers() {
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
}
hipEvent_t Timers::ev() {
    if (next == pool.size()) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        pool.push_back(e);
    }
    return pool[next++];
}
void Timers::begin(int cat) {
    if (!enabled) return;
    hipEvent_t e = ev();
    HIPCHK(hipEventRecord(e, st));
    open_stack.push_back(cat);
    open_ev.push_back(e);
}
void Timers::end(int cat) {
    if (!enabled) return;
    if (open_stack.empty() || open_stack.back() != cat) throw Error("timer nesting error");
    hipEvent_t e = ev();
    HIPCHK(hipEventRecord(e, st));
    pending.push_back({cat, open_ev.back(), e});
    open_stack.pop_back();
    open_ev.pop_back();
}
void Timers::flush() {
    for (auto &p : pending) {
        float ms = 0.f;
        HIPCHK(hipEventSynchronize(p.b));
        HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
        acc[p.cat] += ms * 1e-3;
    }
    pending.clear();
    if (open_stack.empty()) next = 0;
}

void MatOp::apply(const double *x, double *y, Ctx &c) {
    if (!M->sell) build_sell(const_cast<DevCSR &>(*M), c);
    if (timers) timers->begin(T_SPMV);
    spmv(*M, x, y, c);
    if (timers) { timers->end(T_SPMV); timers->spmv_calls++; }
}

// ====================================================== preconditioners ===
void PCNone::apply(const double *x, double *y, Ctx &c) {
    if (x != y) launch_copy(n, x, y, c.st);
}

static void __attribute__((unused)) dummy() {}

PCJacobi::PCJacobi(const DevCSR &M, Ctx &c) {
    type = "jacobi";
    n = M.nrows;
    // diag from host copy of the diagonal (setup only)
    std::vector<int64_t> rp(n + 1);
    std::vector<int32_t> ci(M.nnz);
    std::vector<double> v(M.nnz);
    HIPCHK(hipMemcpyAsync(rp.data(), M.rp.p, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, c.st));
    if (M.nnz) {
        HIPCHK(hipMemcpyAsync(ci.data(), M.ci.p, sizeof(int32_t) * M.nnz, hipMemcpyDeviceToHost, c.st));
        HIPCHK(hipMemcpyAsync(v.data(), M.val.p, sizeof(double) * M.nnz, hipMemcpyDeviceToHost, c.st));
    }
    c.sync();
    std::vector<double> d(n, 1.0);
    for (int64_t i = 0; i < n; ++i) {
        double di = 0.0;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k)
            if (ci[k] == i) { di = v[k]; break; }
        d[i] = (di == 0.0) ? 1.0 : 1.0 / di;
    }
    dinv.alloc(std::max<int64_t>(n, 1));
    HIPCHK(hipMemcpyAsync(dinv.p, d.data(), sizeof(double) * n, hipMemcpyHostToDevice, c.st));
    c.sync();
}
void PCJacobi::apply(const double *x, double *y, Ctx &c) { launch_pointwise_mult(n, x, dinv.p, y, c.st); }


// levels of the strict lower (upper) dependency graph; counting sort into order
static int64_t level_order(int64_t n, const std::vector<int64_t> &rp, const std::vector<int32_t> &ci, bool upper,
                           std::vector<int32_t> &order, std::vector<int64_t> &ptr) {
    std::vector<int32_t> lvl(n, 0);
    int64_t nl = 0;
    if (!upper) {
        for (int64_t i = 0; i < n; ++i) {
            int32_t L = 0;
            for (int64_t k = rp[i]; k < rp[i + 1] && ci[k] < i; ++k) L = std::max(L, lvl[ci[k]] + 1);
            lvl[i] = L;
            nl = std::max<int64_t>(nl, L + 1);
        }
    } else {
        for (int64_t i = n - 1; i >= 0; --i) {
            int32_t L = 0;
            for (int64_t k = rp[i + 1] - 1; k >= rp[i] && ci[k] > i; --k) L = std::max(L, lvl[ci[k]] + 1);
            lvl[i] = L;
            nl = std::max<int64_t>(nl, L + 1);
        }
    }
    ptr.assign(nl + 1, 0);
    for (int64_t i = 0; i < n; ++i) ptr[lvl[i] + 1]++;
    for (int64_t l = 0; l < nl; ++l) ptr[l + 1] += ptr[l];
    order.assign(n, 0);
    std::vector<int64_t> pos(ptr.begin(), ptr.end() - 1);
    for (int64_t i = 0; i < n; ++i) order[pos[lvl[i]]++] = (int32_t)i;
    return nl;
}

// Block-major level groups: rows sorted by (block, level); grp[g] = first row
// of group g, off[b] = first group of block b (PETSc bjacobi block sizes).
// block starts: explicit (bounds) or PETSc's bjacobi sizes
static std::vector<int64_t> block_starts(int64_t n, int64_t nb, const std::vector<int64_t> *bounds) {
    if (bounds) return *bounds;
    std::vector<int64_t> st(nb + 1, 0);
    const int64_t q = n / nb, r = n % nb;
    for (int64_t b = 0; b < nb; ++b) st[b + 1] = st[b] + q + (b < r ? 1 : 0);
    return st;
}

static void block_level_groups(int64_t n, int64_t nb, const std::vector<int64_t> &rp, const std::vector<int32_t> &ci,
                               bool upper, std::vector<int32_t> &order, std::vector<int64_t> &grp,
                               std::vector<int64_t> &off, const std::vector<int64_t> *bounds = nullptr) {
    std::vector<int32_t> lvl(n, 0);
    if (!upper) {
        for (int64_t i = 0; i < n; ++i) {
            int32_t L = 0;
            for (int64_t k = rp[i]; k < rp[i + 1] && ci[k] < i; ++k) L = std::max(L, lvl[ci[k]] + 1);
            lvl[i] = L;
        }
    } else {
        for (int64_t i = n - 1; i >= 0; --i) {
            int32_t L = 0;
            for (int64_t k = rp[i + 1] - 1; k >= rp[i] && ci[k] > i; --k) L = std::max(L, lvl[ci[k]] + 1);
            lvl[i] = L;
        }
    }
    const std::vector<int64_t> bst = block_starts(n, nb, bounds);
    order.clear();
    order.reserve(n);
    grp.clear();
    off.assign(nb + 1, 0);
    int64_t b0 = 0;
    std::vector<int64_t> cnt;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t len = bst[b + 1] - bst[b];
        int32_t nl = 0;
        for (int64_t i = b0; i < b0 + len; ++i) nl = std::max(nl, lvl[i] + 1);
        cnt.assign(nl + 1, 0);
        for (int64_t i = b0; i < b0 + len; ++i) cnt[lvl[i] + 1]++;
        for (int32_t l = 0; l < nl; ++l) cnt[l + 1] += cnt[l];
        off[b] = (int64_t)grp.size();
        const int64_t base = (int64_t)order.size();
        for (int32_t l = 0; l < nl; ++l) grp.push_back(base + cnt[l]);
        order.resize(base + len);
        std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
        for (int64_t i = b0; i < b0 + len; ++i) order[base + pos[lvl[i]]++] = (int32_t)i;
        b0 += len;
    }
    off[nb] = (int64_t)grp.size();
    grp.push_back(n);
}

// Build a level-aligned SELL-64 factor from the factored F: rows in `order`,
// groups = row ranges [grp[g], grp[g+1]) of `order`, goff = first group of
// each block (blockwise) -- padded to whole slices per group.
static void build_tri_sell(const PCILU &P, const std::vector<int64_t> &rp, const std::vector<int64_t> &dg,
                           const std::vector<int32_t> &order, const std::vector<int64_t> &grp,
                           const std::vector<int64_t> *goff, bool upper, TriSELL &T, Ctx &c) {
    const int64_t ng = (int64_t)grp.size() - 1;
    std::vector<int32_t> srow, slen;
    std::vector<int64_t> sl_len;  // 64 * L per slice
    T.gslice_h.assign(ng + 1, 0);
    for (int64_t g = 0; g < ng; ++g) {
        T.gslice_h[g] = (int64_t)sl_len.size();
        for (int64_t r = grp[g]; r < grp[g + 1]; r += 64) {
            int32_t L = 0;
            for (int l = 0; l < 64; ++l) {
                const int64_t rr = r + l;
                if (rr < grp[g + 1]) {
                    const int64_t i = order[rr];
                    const int32_t len = (int32_t)(upper ? rp[i + 1] - dg[i] - 1 : dg[i] - rp[i]);
                    srow.push_back((int32_t)i);
                    slen.push_back(len);
                    L = std::max(L, len);
                } else {
                    srow.push_back(-1);
                    slen.push_back(0);
                }
            }
            sl_len.push_back(64 * (int64_t)L);
        }
    }
    T.gslice_h[ng] = (int64_t)sl_len.size();
    T.ngroups = ng;
    T.nslices = (int64_t)sl_len.size();
    std::vector<int64_t> sptr(T.nslices + 1, 0);
    for (int64_t s = 0; s < T.nslices; ++s) sptr[s + 1] = sptr[s] + sl_len[s];
    auto up64 = [&](DBuf<int64_t> &d, const std::vector<int64_t> &v) {
        d.alloc(std::max<size_t>(v.size(), 1));
        if (!v.empty()) HIPCHK(hipMemcpyAsync(d.p, v.data(), sizeof(int64_t) * v.size(), hipMemcpyHostToDevice, c.st));
    };
    auto up32 = [&](DBuf<int32_t> &d, const std::vector<int32_t> &v) {
        d.alloc(std::max<size_t>(v.size(), 1));
        if (!v.empty()) HIPCHK(hipMemcpyAsync(d.p, v.data(), sizeof(int32_t) * v.size(), hipMemcpyHostToDevice, c.st));
    };
    up64(T.sptr, sptr);
    up64(T.gslice, T.gslice_h);
    up32(T.slot_row, srow);
    up32(T.slot_len, slen);
    T.blockwise = goff != nullptr;
    if (goff) {
        up64(T.goff, *goff);
        T.nblocks = (int64_t)goff->size() - 1;
    }
    T.col.alloc(std::max<int64_t>(sptr.back(), 1));
    T.val.alloc(std::max<int64_t>(sptr.back(), 1));
    if (upper) T.sdinv.alloc(std::max<int64_t>(T.nslices * 64, 1));
    launch_tri_fill(T.nslices, T.slot_row.p, T.slot_len.p, P.F.rp.p, P.F.ci.p, P.F.val.p, P.diag.p, P.dinv.p,
                    upper ? 1 : 0, T.sptr.p, T.col.p, T.val.p, upper ? T.sdinv.p : nullptr, c.st);
    HIPCHK(hipGetLastError());
    c.sync();
}

// LDS-kernel stream layout (kernels.hip, "LDS sweep stream layout"): per block
// the lanes per row (1, 2 or 4) that fit every lane's share of the block's
// longest row into the kernel's register window; slices of 64 / LPR rows of
// one level; one header entry per lane.
static void build_lds_tri(const PCILU &P, int64_t n, int64_t nb, int force_lpr, int max_lpr,
                          const std::vector<int64_t> &rp,
                          const std::vector<int64_t> &dg, const std::vector<int32_t> &order,
                          const std::vector<int64_t> &grp, const std::vector<int64_t> &goff, bool upper, LdsTri &D,
                          Ctx &c, const std::vector<int32_t> *posof = nullptr,
                          const std::vector<int32_t> *row_lo = nullptr, const std::vector<int32_t> *near_len = nullptr,
                          std::vector<int64_t> *blk_maxsl = nullptr) {
    const int64_t ng = (int64_t)grp.size() - 1, nblk = (int64_t)goff.size() - 1;
    const int W = ilu_lds_lane_entries();
    auto rlen = [&](int64_t i) -> int64_t {
        if (near_len) return (*near_len)[i];  // ring sweep: the near entries only
        return upper ? rp[i + 1] - dg[i] - 1 : dg[i] - rp[i];
    };
    std::vector<int32_t> lpr(nblk, 1), s_start, s_n, s_lpr;
    std::vector<int64_t> gsl(ng + 1, 0), sptr(1, 0);
    for (int64_t b = 0; b < nblk; ++b) {
        // lanes per row: the fewest that fit the longest row's per-lane share
        // into the kernel's register window (measured at N=59: 2 or 4 lanes
        // on short rows cost more in extra slices and headers than they gain)
        int64_t mx = 0;
        for (int64_t r = grp[goff[b]]; r < grp[goff[b + 1]]; ++r) mx = std::max(mx, rlen(order[r]));
        // (the y-resident sweep, max_lpr 16: its y gathers miss LDS, so an
        // in-level reload of a long row's tail costs an HBM round trip per
        // level; up to 16 lanes keep every entry in the prefetched window)
        // (capping the lanes so the widest level fits one slice per wave was
        // measured slower: FE 3-D N=12 53 -> 44 it/s, N=20 unchanged)
        int l = 1;
        while (l < max_lpr && (mx + l - 1) / l > W) l *= 2;
        if (force_lpr) {
            // pls.sweep_lpr: the sweep kernels are instantiated for 1/2/4 lanes per
            // row (LDS) and 1/2/4/8/16 (y-resident); anything else would run slices
            // under the wrong template and silently corrupt the apply
            if (force_lpr < 1 || force_lpr > max_lpr || (force_lpr & (force_lpr - 1)))
                throw Error("pls.sweep_lpr " + std::to_string(force_lpr) + " not supported by this sweep (allowed: 1.." +
                            std::to_string(max_lpr) + ", powers of two)");
            l = force_lpr;
        }
        lpr[b] = l;
        const int64_t per = 64 / l;
        if (posof) {
            // ring sweep: lanes per row chosen per slice (rows sorted longest first
            // inside each level): the fewest that keep every lane's share within the
            // register window, so short-row slices hold more rows and a level needs
            // fewer slices than the workgroup has waves (no in-level reloads)
            for (int64_t g = goff[b]; g < goff[b + 1]; ++g) {
                gsl[g] = (int64_t)s_start.size();
                for (int64_t r0 = grp[g]; r0 < grp[g + 1];) {
                    const int WR = ilu_ring_lane_entries();
                    int ls = force_lpr ? force_lpr : 1;  // pls.sweep_lpr pins it
                    int64_t r1 = 0, mxs = 0;
                    for (;;) {
                        r1 = std::min(grp[g + 1], r0 + 64 / ls);
                        mxs = 0;
                        for (int64_t r = r0; r < r1; ++r) mxs = std::max(mxs, rlen(order[r]));
                        if ((mxs + ls - 1) / ls <= WR || ls >= 32 || force_lpr) break;
                        ls *= 2;
                    }
                    s_start.push_back((int32_t)r0);
                    s_n.push_back((int32_t)(r1 - r0));
                    s_lpr.push_back(ls);
                    // lane-major entries, a multiple of the slot (WR + 1) per lane (header included)
                    sptr.push_back(sptr.back() + 64 * ((((mxs + ls - 1) / ls + 1) + WR) / (WR + 1) * (WR + 1)));
                    lpr[b] = std::max(lpr[b], ls);
                    r0 = r1;
                }
            }
            continue;
        }
        for (int64_t g = goff[b]; g < goff[b + 1]; ++g) {
            gsl[g] = (int64_t)s_start.size();
            for (int64_t r0 = grp[g]; r0 < grp[g + 1]; r0 += per) {
                const int64_t r1 = std::min(grp[g + 1], r0 + per);
                int64_t L = 0;
                for (int64_t r = r0; r < r1; ++r) L = std::max(L, (rlen(order[r]) + l - 1) / l);
                s_start.push_back((int32_t)r0);
                s_n.push_back((int32_t)(r1 - r0));
                s_lpr.push_back(l);
                sptr.push_back(sptr.back() + 64 * (L + 1));
            }
        }
    }
    gsl[ng] = (int64_t)s_start.size();
    const int64_t ns = (int64_t)s_start.size();
    if (blk_maxsl) {  // per block: the most slices any level has (max over both triangles)
        blk_maxsl->resize(nblk, 0);
        for (int64_t b = 0; b < nblk; ++b)
            for (int64_t g = goff[b]; g < goff[b + 1]; ++g) (*blk_maxsl)[b] = std::max((*blk_maxsl)[b], gsl[g + 1] - gsl[g]);
    }
    if (c.ilu_view >= 2 && !posof) {
        // per block: levels, slices beyond the 16 waves (run inline with dependent
        // loads), slices whose lanes hold more than the W prefetched entries
        int64_t worst_inline = 0, worst_lev = 0, worst_long = 0, wmax = 0, b_inl = 0;
        for (int64_t b = 0; b < nblk; ++b) {
            int64_t inl = 0, lng = 0;
            for (int64_t g = goff[b]; g < goff[b + 1]; ++g) {
                const int64_t s = gsl[g + 1] - gsl[g];
                wmax = std::max(wmax, s);
                inl += std::max<int64_t>(0, s - 16);
                for (int64_t k = gsl[g]; k < gsl[g + 1]; ++k) lng += (sptr[k + 1] - sptr[k]) / 64 - 1 > W;
            }
            if (inl > worst_inline) { worst_inline = inl; b_inl = b; }
            worst_lev = std::max(worst_lev, goff[b + 1] - goff[b]);
            worst_long = std::max(worst_long, lng);
        }
        fprintf(stderr, "[pls ilu lds %s] blocks %lld: max levels %lld, max slices per level %lld, inline slices "
                "(beyond 16 waves) max %lld (block %lld), slices with > %d entries per lane max %lld\n",
                upper ? "U" : "L", (long long)nblk, (long long)worst_lev, (long long)wmax, (long long)worst_inline,
                (long long)b_inl, W, (long long)worst_long);
    }
    auto up = [&](auto &d, const auto &v) {
        d.alloc(std::max<size_t>(v.size(), 1));
        if (!v.empty())
            HIPCHK(hipMemcpyAsync(d.p, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice, c.st));
    };
    DBuf<int32_t> d_start, d_n, d_lpr, d_order;
    up(D.sptr, sptr);
    up(D.gslice, gsl);
    up(D.lpr, lpr);
    up(d_start, s_start);
    up(d_n, s_n);
    up(d_lpr, s_lpr);
    up(d_order, order);
    D.col.alloc(std::max<int64_t>(sptr.back(), 1));
    D.val.alloc(std::max<int64_t>(sptr.back(), 1));
    DBuf<int32_t> d_posof, d_lo;
    if (posof) up(d_posof, *posof);
    if (row_lo) up(d_lo, *row_lo);
    launch_lds_fill(ns, d_start.p, d_n.p, d_lpr.p, d_order.p, P.F.rp.p, P.F.ci.p, P.F.val.p, P.diag.p, P.dinv.p,
                    upper ? 1 : 0, n, nb, D.sptr.p, D.col.p, D.val.p, c.st, /*wide headers: y-resident sweep*/ max_lpr > 4,
                    posof ? d_posof.p : nullptr, row_lo ? d_lo.p : nullptr, P.bstart_h.empty() ? nullptr : P.bstart.p);
    HIPCHK(hipGetLastError());
    c.sync();
    if (posof) {  // ring sweep: slice starts carry log2(lanes per row) in bits 0-2
        for (int64_t k = 0; k < ns; ++k) {
            int l2 = 0;
            while ((1 << l2) < s_lpr[k]) ++l2;
            sptr[k] |= l2;
        }
        HIPCHK(hipMemcpyAsync(D.sptr.p, sptr.data(), sizeof(int64_t) * sptr.size(), hipMemcpyHostToDevice, c.st));
        c.sync();
    }
}

void TriSELL::apply(const double *b, double *y, Ctx &c) const {
    const double *dv = sdinv.p;
    if (blockwise) {
        launch_tri_blocks(nblocks, goff.p, gslice.p, sptr.p, slot_row.p, slot_len.p, col.p, val.p, dv, b, y, c.st);
        return;
    }
    for (int64_t g = 0; g < ngroups; ++g)
        launch_tri_group(gslice_h[g], gslice_h[g + 1], sptr.p, slot_row.p, slot_len.p, col.p, val.p, dv, b, y, c.st);
}

// Profile (envelope) pattern of M with M's values and explicit zeros.
static void envelope_csr(const DevCSR &M, DevCSR &E, Ctx &c) {
    const int64_t n = M.nrows;
    std::vector<int64_t> rp(n + 1);
    std::vector<int32_t> ci(M.nnz);
    std::vector<double> v(M.nnz);
    HIPCHK(hipMemcpyAsync(rp.data(), M.rp.p, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, c.st));
    if (M.nnz) {
        HIPCHK(hipMemcpyAsync(ci.data(), M.ci.p, sizeof(int32_t) * M.nnz, hipMemcpyDeviceToHost, c.st));
        HIPCHK(hipMemcpyAsync(v.data(), M.val.p, sizeof(double) * M.nnz, hipMemcpyDeviceToHost, c.st));
    }
    c.sync();
    std::vector<int64_t> erp(n + 1, 0), lo(n), hi(n);
    int64_t hmax = -1;
    for (int64_t i = 0; i < n; ++i) {
        int64_t a = i, b = i;
        if (rp[i + 1] > rp[i]) {
            a = std::min<int64_t>(a, ci[rp[i]]);
            b = std::max<int64_t>(b, ci[rp[i + 1] - 1]);
        }
        hmax = std::max(hmax, b);
        lo[i] = a;
        hi[i] = std::max<int64_t>(hmax, i);
        erp[i + 1] = erp[i] + (hi[i] - lo[i] + 1);
        if (hi[i] - lo[i] + 1 > ilu0_max_row())
            throw Error("lu: profile row longer than " + std::to_string(ilu0_max_row()) +
                        " entries; use ilu/bjacobi");
    }
    if (erp[n] > 400000000LL) throw Error("lu: profile fill exceeds 4e8 entries; use ilu/bjacobi on the device");
    std::vector<int32_t> eci(erp[n]);
    std::vector<double> ev(erp[n], 0.0);
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t j = lo[i]; j <= hi[i]; ++j) eci[erp[i] + (j - lo[i])] = (int32_t)j;
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) ev[erp[i] + (ci[k] - lo[i])] = v[k];
    }
    upload_csr(E, n, n, erp.data(), eci.data(), ev.data(), c);
}

// Ring sweep tables of one triangle: block-local level-order positions of the
// rows (posof), and level-aligned chunks of at most ilu_ring_chunk() positions.
// A row's dependency at position q is "near" when q >= row_lo[row] = (end of
// the row's chunk) - ilu_ring_slots(): still in the ring while the row runs.
// Far ones go to a CSR over positions, applied when the row's chunk loads.
static void ring_tables(int64_t n, int64_t nb, const std::vector<int32_t> &order, const std::vector<int64_t> &grp,
                        const std::vector<int64_t> &goff, const std::vector<int64_t> &rp, const std::vector<int32_t> &ci,
                        const std::vector<int64_t> &dg, const std::vector<double> &fv, bool upper,
                        std::vector<int32_t> &posof, std::vector<int32_t> &row_lo, std::vector<int32_t> &near_len,
                        RingTri &T, Ctx &c, const std::vector<int64_t> *bounds = nullptr) {
    const std::vector<int64_t> bst = block_starts(n, nb, bounds);
    const int64_t C = ilu_ring_chunk(), R = ilu_ring_slots();
    posof.assign(n, 0);
    row_lo.assign(n, 0);
    near_len.assign(n, 0);
    std::vector<int64_t> coff(nb + 1, 0), cg, cp;
    int64_t b0 = 0;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t len = bst[b + 1] - bst[b];
        for (int64_t k = b0; k < b0 + len; ++k) posof[order[k]] = (int32_t)(k - b0);
        coff[b] = (int64_t)cg.size();
        for (int64_t g = goff[b]; g < goff[b + 1];) {
            const int64_t c0 = grp[g] - b0;
            int64_t e = g + 1;
            while (e < goff[b + 1] && grp[e + 1] - b0 - c0 <= C) ++e;
            cg.push_back(g);
            cp.push_back(c0);
            cp.push_back(grp[e] - b0);
            for (int64_t k = grp[g]; k < grp[e]; ++k) row_lo[order[k]] = (int32_t)(grp[e] - b0 - R);
            g = e;
        }
        b0 += len;
    }
    coff[nb] = (int64_t)cg.size();
    // far dependencies, by position (b0 + p), in the row's entry order
    std::vector<int64_t> frp(n + 1, 0);
    std::vector<int32_t> fcol;
    std::vector<double> fval;
    for (int64_t k = 0; k < n; ++k) {
        const int64_t i = order[k];
        const int64_t s0 = upper ? dg[i] + 1 : rp[i], s1 = upper ? rp[i + 1] : dg[i];
        int64_t near = 0;
        for (int64_t e = s0; e < s1; ++e) {
            const int32_t pc = posof[ci[e]];
            if (pc >= row_lo[i]) {
                ++near;
            } else {
                fcol.push_back(pc);
                fval.push_back(fv[e]);
            }
        }
        near_len[i] = (int32_t)near;
        frp[k + 1] = (int64_t)fcol.size();
    }
    T.nfar = (int64_t)fcol.size();
    auto up = [&](auto &d, const auto &v) {
        d.alloc(std::max<size_t>(v.size(), 1));
        if (!v.empty()) HIPCHK(hipMemcpyAsync(d.p, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice, c.st));
    };
    up(T.coff, coff);
    up(T.cg, cg);
    up(T.cp, cp);
    up(T.ord, order);
    up(T.frp, frp);
    up(T.fcol, fcol);
    up(T.fval, fval);
    c.sync();
}

// Chain-sweep stream of one triangle (kernels.hip, "chain sweep"): per block
// the fewest lanes per row (1..ilu_chain_max_lpr(), powers of two) that keep
// every lane's share of the block's longest row within 7 entries -- the LDS
// sweep's rule, so blocks whose rows fit 4 lanes get the LDS sweep's lanes and
// sums -- then per level steps of 16 / lpr rows in the level's row order, and
// slices of up to 4 consecutive steps (step q on lanes 16q .. 16q + 15).
// Returns the step count, or -1 when a row does not fit (fv / dinv empty: a
// dry run that only counts).
// Window-sweep tables of one triangle of the (block-truncated) factors F (rp,
// ci, fv, diagonal positions dg): per block, windows of 64 consecutive rows;
// per window the rows' entries outside the window on the solved side (SELL,
// [k][lane], block-local columns) and the inverse of the window's triangle --
// unit lower (I + L_ww) or upper with the diagonal (U_ww) -- by row-wise
// substitution in double precision without contraction, stored [k][lane].
// Largest number of off-window entries of a row (the kernel's limit: ilu_window_max_entries())
static void window_max_entries_lu(int64_t nblk, const std::vector<int64_t> &bst, const std::vector<int64_t> &rp,
                                  const std::vector<int32_t> &ci, const std::vector<int64_t> &dg, int &eL, int &eU) {
    int64_t kml = 0, kmu = 0;
    for (int64_t b = 0; b < nblk; ++b)
        for (int64_t i = bst[b]; i < bst[b + 1]; ++i) {
            const int64_t w0 = bst[b] + (i - bst[b]) / 64 * 64, w1 = std::min<int64_t>(w0 + 64, bst[b + 1]);
            int64_t kl = 0, ku = 0;
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                kl += ci[k] < w0;
                ku += ci[k] >= w1;
            }
            kml = std::max(kml, kl);
            kmu = std::max(kmu, ku);
        }
    eL = (int)kml;
    eU = (int)kmu;
}
static int64_t window_max_entries(int64_t nblk, const std::vector<int64_t> &bst, const std::vector<int64_t> &rp,
                                  const std::vector<int32_t> &ci, const std::vector<int64_t> &dg) {
    int eL = 0, eU = 0;
    window_max_entries_lu(nblk, bst, rp, ci, dg, eL, eU);
    return std::max(eL, eU);
}
// Farthest dependency of a row in rows (|i - c| over the off-diagonal entries;
// the ring variant's limit: ilu_window_ring_rows() - 64)
static int64_t window_max_reach(int64_t n, const std::vector<int64_t> &rp, const std::vector<int32_t> &ci) {
    int64_t r = 0;
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) r = std::max<int64_t>(r, std::abs(i - (int64_t)ci[k]));
    return r;
}

static void build_window_tri(int64_t nblk, const std::vector<int64_t> &bst, const std::vector<int64_t> &rp,
                             const std::vector<int32_t> &ci, const std::vector<int64_t> &dg,
                             const std::vector<double> &fv, bool upper, WinTri &W, Ctx &c) {
    std::vector<int64_t> wfirst(nblk + 1, 0);
    for (int64_t b = 0; b < nblk; ++b) wfirst[b + 1] = wfirst[b] + (bst[b + 1] - bst[b] + 63) / 64;
    const int64_t nw = wfirst[nblk];
    std::vector<int64_t> wrow(nw), wend(nw);  // first row, end row of each window
    for (int64_t b = 0; b < nblk; ++b)
        for (int64_t w = wfirst[b]; w < wfirst[b + 1]; ++w) {
            wrow[w] = bst[b] + (w - wfirst[b]) * 64;
            wend[w] = std::min<int64_t>(wrow[w] + 64, bst[b + 1]);
        }
    auto off_range = [&](int64_t i, int64_t w, int64_t &k0, int64_t &k1) {  // entries of row i outside window w
        if (!upper) {
            k0 = rp[i];
            k1 = k0;
            while (k1 < dg[i] && ci[k1] < wrow[w]) ++k1;
        } else {
            k1 = rp[i + 1];
            k0 = k1;
            while (k0 > dg[i] + 1 && ci[k0 - 1] >= wend[w]) --k0;
        }
    };
    std::vector<int64_t> woff(nw + 1, 0);
    for (int64_t w = 0; w < nw; ++w) {
        int64_t K = 0;
        for (int64_t i = wrow[w]; i < wend[w]; ++i) {
            int64_t k0, k1;
            off_range(i, w, k0, k1);
            K = std::max(K, k1 - k0);
        }
        woff[w + 1] = woff[w] + K * 64;
    }
    // (the staging copies read a fixed number of entries past a window's start: padding at the end)
    std::vector<int32_t> rec(3 * (woff[nw] + ilu_window_stream_pad()), 0);
    std::vector<double> tinv((size_t)std::max<int64_t>(nw, 1) * 4096, 0.0);
    auto put = [&](int64_t e, int32_t col, double v) {
        std::memcpy(&rec[3 * e], &v, 8);
        rec[3 * e + 2] = col;
    };
    amgh::parallel_rows(nw, amgh::setup_threads(), [&](int, int64_t w0, int64_t w1) {
        std::vector<double> T(64 * 64), X(64 * 64);
        for (int64_t w = w0; w < w1; ++w) {
            int64_t b = std::upper_bound(wfirst.begin(), wfirst.end(), w) - wfirst.begin() - 1;
            const int64_t r0 = wrow[w], m = wend[w] - r0, base = bst[b];
            std::fill(T.begin(), T.end(), 0.0);
            for (int64_t i = r0; i < wend[w]; ++i) {
                const int lane = (int)(i - r0);
                int64_t k0, k1;
                off_range(i, w, k0, k1);
                for (int64_t k = k0; k < k1; ++k) put(woff[w] + (k - k0) * 64 + lane, (int32_t)(ci[k] - base), fv[k]);
                // the window's triangle, row-major T[i][j]
                if (!upper) {
                    T[lane * 64 + lane] = 1.0;
                    for (int64_t k = k1; k < dg[i]; ++k) T[lane * 64 + (ci[k] - r0)] = fv[k];
                } else {
                    for (int64_t k = dg[i]; k < k0; ++k) T[lane * 64 + (ci[k] - r0)] = fv[k];
                }
            }
            std::fill(X.begin(), X.end(), 0.0);
            if (!upper) {  // X = T^-1, T unit lower: row i of X from rows j < i
                for (int64_t i = 0; i < m; ++i) {
                    X[i * 64 + i] = 1.0;
                    for (int64_t j = 0; j < i; ++j) {
                        double s = 0.0;
                        for (int64_t k = j; k < i; ++k) s += T[i * 64 + k] * X[k * 64 + j];
                        X[i * 64 + j] = -s;
                    }
                }
            } else {  // T upper with its diagonal: rows from the last
                for (int64_t i = m - 1; i >= 0; --i) {
                    const double d = T[i * 64 + i];
                    X[i * 64 + i] = 1.0 / d;
                    for (int64_t j = i + 1; j < m; ++j) {
                        double s = 0.0;
                        for (int64_t k = i + 1; k <= j; ++k) s += T[i * 64 + k] * X[k * 64 + j];
                        X[i * 64 + j] = -s / d;
                    }
                }
            }
            for (int64_t i = 0; i < 64; ++i)  // column pairs: lane i loads X[i][k], X[i][k + 1] at once
                for (int64_t k = 0; k < 64; ++k) tinv[(size_t)w * 4096 + (k >> 1) * 128 + i * 2 + (k & 1)] = X[i * 64 + k];
        }
    });
    W.nwin = nw;
    W.woff.alloc(nw + 1);
    W.rec.alloc(rec.size());
    W.tinv.alloc(tinv.size());
    HIPCHK(hipMemcpyAsync(W.woff.p, woff.data(), sizeof(int64_t) * (nw + 1), hipMemcpyHostToDevice, c.st));
    HIPCHK(hipMemcpyAsync(W.rec.p, rec.data(), sizeof(int32_t) * rec.size(), hipMemcpyHostToDevice, c.st));
    HIPCHK(hipMemcpyAsync(W.tinv.p, tinv.data(), sizeof(double) * tinv.size(), hipMemcpyHostToDevice, c.st));
    c.sync();
}

// Super-window sweep tables of one triangle (kernels.hip, k_ilu_blocks_swin)
// for blocks too long for LDS.  Rows are cut into windows of 64 (from the
// block's first row, as build_window_tri), consecutive windows into
// super-windows in processing order (ascending for L, descending for U) as
// long as their staged data -- the packed window inverses (2,080 doubles) and
// the near streams -- fit ilu_swin_lds_budget() (at most 8 windows).  A row's
// entries on the solved side split three ways: in its own window (into the
// window's triangle, inverted as build_window_tri does), near (in its super-
// window, another window: SELL [k][lane], column = row - the super-window's
// first row, read from LDS) and far (before the super-window: SELL, block-
// local row, read from the block solution in global memory).  Padding entries
// carry column 0 and value 0.
static void build_swin_tri(int64_t nblk, const std::vector<int64_t> &bst, const std::vector<int64_t> &rp,
                           const std::vector<int32_t> &ci, const std::vector<int64_t> &dg,
                           const std::vector<double> &fv, bool upper, SwinTri &W, Ctx &c) {
    std::vector<int64_t> wfirst(nblk + 1, 0);
    for (int64_t b = 0; b < nblk; ++b) wfirst[b + 1] = wfirst[b] + (bst[b + 1] - bst[b] + 63) / 64;
    const int64_t nw = wfirst[nblk];
    std::vector<int64_t> wrow(nw), wend(nw), wblk(nw);  // first / end row (global), block
    for (int64_t b = 0; b < nblk; ++b)
        for (int64_t w = wfirst[b]; w < wfirst[b + 1]; ++w) {
            wrow[w] = bst[b] + (w - wfirst[b]) * 64;
            wend[w] = std::min<int64_t>(wrow[w] + 64, bst[b + 1]);
            wblk[w] = b;
        }
    // solved-side entries of row i: [s0, s1) in column order
    auto side = [&](int64_t i, int64_t &s0, int64_t &s1) {
        if (!upper) {
            s0 = rp[i];
            s1 = dg[i];
        } else {
            s0 = dg[i] + 1;
            s1 = rp[i + 1];
        }
    };
    // counts of row i's near / far entries for a super-window spanning rows [lo, hi) (global)
    auto counts = [&](int64_t i, int64_t w, int64_t lo, int64_t hi, int64_t &nn, int64_t &nf) {
        int64_t s0, s1;
        side(i, s0, s1);
        nn = nf = 0;
        for (int64_t k = s0; k < s1; ++k) {
            const int64_t cc = ci[k];
            if (cc >= wrow[w] && cc < wend[w]) continue;  // own window: the triangle
            if (cc >= lo && cc < hi) ++nn;
            else ++nf;
        }
    };
    auto win_near = [&](int64_t w, int64_t lo, int64_t hi) {  // the window's near entries per lane (max over rows)
        int64_t K = 0;
        for (int64_t i = wrow[w]; i < wend[w]; ++i) {
            int64_t nn, nf;
            counts(i, w, lo, hi, nn, nf);
            K = std::max(K, nn);
        }
        return K;
    };
    const int64_t budget = ilu_swin_lds_budget(), TRI = 2080;
    // super-windows, per block in processing order (greedy)
    std::vector<int64_t> bsw(nblk + 1, 0), sw;  // sw: 4 per super-window
    std::vector<int64_t> swof(nw, 0);           // window -> super-window
    int64_t max_stage = 0;
    for (int64_t b = 0; b < nblk; ++b) {
        const int64_t W0 = wfirst[b], W1 = wfirst[b + 1];
        int64_t k = 0;
        const int64_t nwb = W1 - W0;
        while (k < nwb) {
            const int64_t first = upper ? W1 - 1 - k : W0 + k;
            int64_t cnt = 0, bytes = 0;
            for (;;) {
                if (k + cnt >= nwb || cnt == 8) break;
                const int64_t w = upper ? W1 - 1 - (k + cnt) : W0 + k + cnt;
                // the super-window's rows if w joins: [lo, hi)
                const int64_t lo = upper ? wrow[w] : wrow[first], hi = upper ? wend[first] : wend[w];
                const int64_t add = TRI * 8 + win_near(w, lo, hi) * 64 * 12;
                if (cnt > 0 && bytes + add > budget) break;
                bytes += add;
                ++cnt;
            }
            const int64_t last = upper ? W1 - 1 - (k + cnt - 1) : W0 + k + cnt - 1;
            const int64_t wlo = std::min(first, last);
            sw.push_back(wlo);  // first window (ascending storage)
            sw.push_back(cnt);
            sw.push_back(wrow[wlo] - bst[b]);
            sw.push_back(wend[std::max(first, last)] - bst[b]);
            for (int64_t w = wlo; w < wlo + cnt; ++w) swof[w] = (int64_t)sw.size() / 4 - 1;
            max_stage = std::max(max_stage, bytes);
            k += cnt;
        }
        bsw[b + 1] = (int64_t)sw.size() / 4;
    }
    const int64_t nsw = (int64_t)sw.size() / 4;
    // per-window stream sizes
    std::vector<int64_t> wnear(nw + 1, 0), wfar(nw + 1, 0);
    {
        std::vector<int64_t> kn(nw), kf(nw);
        amgh::parallel_rows(nw, amgh::setup_threads(), [&](int, int64_t w0, int64_t w1) {
            for (int64_t w = w0; w < w1; ++w) {
                const int64_t s = swof[w], b = wblk[w];
                const int64_t lo = bst[b] + sw[4 * s + 2], hi = bst[b] + sw[4 * s + 3];
                int64_t a = 0, f = 0;
                for (int64_t i = wrow[w]; i < wend[w]; ++i) {
                    int64_t nn, nf;
                    counts(i, w, lo, hi, nn, nf);
                    a = std::max(a, nn);
                    f = std::max(f, nf);
                }
                kn[w] = a;
                kf[w] = f;
            }
        });
        for (int64_t w = 0; w < nw; ++w) {
            wnear[w + 1] = wnear[w] + kn[w] * 64;
            wfar[w + 1] = wfar[w] + kf[w] * 64;
        }
    }
    std::vector<int32_t> ncol(std::max<int64_t>(wnear[nw], 1), 0), fcol(std::max<int64_t>(wfar[nw], 1), 0);
    std::vector<double> nval(ncol.size(), 0.0), fval(fcol.size(), 0.0), tinv((size_t)std::max<int64_t>(nw, 1) * TRI, 0.0);
    amgh::parallel_rows(nw, amgh::setup_threads(), [&](int, int64_t w0, int64_t w1) {
        std::vector<double> T(64 * 64), X(64 * 64);
        for (int64_t w = w0; w < w1; ++w) {
            const int64_t s = swof[w], b = wblk[w], base = bst[b];
            const int64_t lo = base + sw[4 * s + 2], hi = base + sw[4 * s + 3];
            const int64_t r0 = wrow[w], m = wend[w] - r0;
            std::fill(T.begin(), T.end(), 0.0);
            for (int64_t i = r0; i < wend[w]; ++i) {
                const int lane = (int)(i - r0);
                int64_t s0, s1, qn = 0, qf = 0;
                side(i, s0, s1);
                if (!upper) T[lane * 64 + lane] = 1.0;
                for (int64_t k = s0; k < s1; ++k) {
                    const int64_t cc = ci[k];
                    if (cc >= r0 && cc < wend[w]) {
                        T[lane * 64 + (cc - r0)] = fv[k];
                    } else if (cc >= lo && cc < hi) {
                        ncol[wnear[w] + qn * 64 + lane] = (int32_t)(cc - lo);
                        nval[wnear[w] + qn * 64 + lane] = fv[k];
                        ++qn;
                    } else {
                        fcol[wfar[w] + qf * 64 + lane] = (int32_t)(cc - base);
                        fval[wfar[w] + qf * 64 + lane] = fv[k];
                        ++qf;
                    }
                }
                if (upper) T[lane * 64 + lane] = fv[dg[i]];
            }
            std::fill(X.begin(), X.end(), 0.0);
            if (!upper) {  // X = T^-1, T unit lower
                for (int64_t i = 0; i < m; ++i) {
                    X[i * 64 + i] = 1.0;
                    for (int64_t j = 0; j < i; ++j) {
                        double acc = 0.0;
                        for (int64_t k = j; k < i; ++k) acc += T[i * 64 + k] * X[k * 64 + j];
                        X[i * 64 + j] = -acc;
                    }
                }
            } else {  // T upper with its diagonal
                for (int64_t i = m - 1; i >= 0; --i) {
                    const double d = T[i * 64 + i];
                    X[i * 64 + i] = 1.0 / d;
                    for (int64_t j = i + 1; j < m; ++j) {
                        double acc = 0.0;
                        for (int64_t k = i + 1; k <= j; ++k) acc += T[i * 64 + k] * X[k * 64 + j];
                        X[i * 64 + j] = -acc / d;
                    }
                }
            }
            // packed by column k: L -- rows k..63 at 64k - k(k-1)/2 + (row - k); U -- rows 0..k at k(k+1)/2 + row
            double *t = &tinv[(size_t)w * TRI];
            for (int64_t k = 0; k < 64; ++k) {
                if (!upper)
                    for (int64_t i = k; i < 64; ++i) t[64 * k - k * (k - 1) / 2 + (i - k)] = X[i * 64 + k];
                else
                    for (int64_t i = 0; i <= k; ++i) t[k * (k + 1) / 2 + i] = X[i * 64 + k];
            }
        }
    });
    auto up = [&](auto &d, const auto &v) {
        d.alloc(std::max<size_t>(v.size(), 1));
        if (!v.empty()) HIPCHK(hipMemcpyAsync(d.p, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice, c.st));
    };
    up(W.bsw, bsw);
    up(W.sw, sw);
    up(W.wnear, wnear);
    up(W.wfar, wfar);
    up(W.ncol, ncol);
    up(W.nval, nval);
    up(W.fcol, fcol);
    up(W.fval, fval);
    up(W.tinv, tinv);
    c.sync();
    W.nwin = nw;
    W.nsw = nsw;
    W.lds_bytes = 576 * 8 + max_stage;  // (the kernel's rows + broadcast slots, then the staged data)
}

static int64_t build_chain_tri(int64_t nblk, const std::vector<int64_t> &bst, const std::vector<int64_t> &rp,
                               const std::vector<int32_t> &ci, const std::vector<int64_t> &dg,
                               const std::vector<double> &fv, const std::vector<double> &dinv,
                               const std::vector<int32_t> &order, const std::vector<int64_t> &grp,
                               const std::vector<int64_t> &goff, bool upper, ChainTri *D, Ctx &c) {
    const int W = ilu_lds_lane_entries(), LMAX = ilu_chain_max_lpr();
    const int32_t PAD = (1 << 18) - 1;  // kernels.hip SW_ROW_PAD
    auto rlen = [&](int64_t i) -> int64_t { return upper ? rp[i + 1] - dg[i] - 1 : dg[i] - rp[i]; };
    const bool dry = D == nullptr;
    std::vector<int64_t> base(nblk, 0), nsl(nblk, 0), soff(nblk, 0);
    std::vector<int32_t> szs, lpr(nblk, 1), col;
    std::vector<double> val;
    int64_t total = 0;
    for (int64_t b = 0; b < nblk; ++b) {
        const int64_t b0 = bst[b];
        int64_t mx = 0;
        for (int64_t r = grp[goff[b]]; r < grp[goff[b + 1]]; ++r) mx = std::max(mx, rlen(order[r]));
        int l = 1;
        while (l < LMAX && (mx + l - 1) / l > W) l *= 2;
        if ((mx + l - 1) / l > W) return -1;
        lpr[b] = l;
        const int64_t per = 16 / l;
        // steps: [first row, end row) in `order` positions, a level's rows cut every `per`
        std::vector<std::pair<int64_t, int64_t>> steps;
        for (int64_t g = goff[b]; g < goff[b + 1]; ++g)
            for (int64_t r0 = grp[g]; r0 < grp[g + 1]; r0 += per) steps.push_back({r0, std::min(grp[g + 1], r0 + per)});
        total += (int64_t)steps.size();
        if (dry) continue;
        std::vector<int32_t> sizes;
        base[b] = (int64_t)col.size();
        for (size_t s0 = 0; s0 < steps.size(); s0 += 4) {
            const size_t ns = std::min<size_t>(4, steps.size() - s0);
            // 8 entries per lane (header + 7; the lanes per row keep every share <= 7),
            // unused ones (column 0, value 0): the kernel sums all 7 without masking
            const int L = 8;
            const int64_t nl = 16 * (int64_t)ns, sz = nl * L;
            sizes.push_back((int32_t)(sz | (L == 8 ? 1 : 0)));
            const int64_t at = (int64_t)col.size();
            col.resize(at + sz, 0);
            val.resize(at + sz, 0.0);
            for (int64_t lane = 0; lane < nl; ++lane) col[at + lane * L] = PAD;  // lanes without a row
            for (size_t q = 0; q < ns; ++q) {
                for (int64_t r = steps[s0 + q].first; r < steps[s0 + q].second; ++r) {
                    const int64_t rr = r - steps[s0 + q].first;
                    const int64_t i = order[r];
                    const int64_t src = upper ? dg[i] + 1 : rp[i], len = rlen(i);
                    for (int sub = 0; sub < l; ++sub) {
                        const int64_t mine = len > sub ? (len - sub + l - 1) / l : 0;
                        const int64_t e = at + (16 * (int64_t)q + rr * l + sub) * L;
                        col[e] = (int32_t)(i - b0) | (int32_t)(mine << 18);
                        val[e] = upper ? dinv[i] : 0.0;
                        for (int64_t k = 1; k <= mine; ++k) {
                            const int64_t j = (k - 1) * l + sub;
                            col[e + k] = ci[src + j] - (int32_t)b0;
                            val[e + k] = fv[src + j];
                        }
                    }
                }
            }
        }
        nsl[b] = (int64_t)sizes.size();
        soff[b] = (int64_t)szs.size();
        szs.insert(szs.end(), sizes.begin(), sizes.end());
    }
    if (dry) return total;
    auto up = [&](auto &d, const auto &v) {
        d.alloc(std::max<size_t>(v.size(), 1));
        if (!v.empty()) HIPCHK(hipMemcpyAsync(d.p, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice, c.st));
    };
    up(D->base, base);
    up(D->nsl, nsl);
    up(D->soff, soff);
    up(D->sz, szs);
    up(D->lpr, lpr);
    up(D->col, col);
    up(D->val, val);
    c.sync();
    return total;
}

PCILU::PCILU(const DevCSR &M, int64_t nb, Ctx &c, bool exact_lu, bool lds, int force_lpr, int gmem_mode,
             int ring_mode, bool sgs_factors, const std::vector<int64_t> *bounds) {
    const bool trace = std::getenv("PLS_ILU_TRACE") != nullptr && M.nrows > 100000;
    auto tnow = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double tm0 = tnow();
    auto mark = [&](const char *what) {
        if (!trace) return;
        const double t = tnow();
        fprintf(stderr, "[pcilu n %lld] %s %.3f s\n", (long long)M.nrows, what, t - tm0);
        tm0 = t;
    };
    exact = exact_lu;
    sgs = sgs_factors && !exact_lu;
    allow_lds = lds;
    type = exact ? "lu" : sgs ? "sgs" : (nb > 1 ? "bjacobi" : "ilu");
    n = M.nrows;
    nblocks = exact ? 1 : std::max<int64_t>(1, std::min<int64_t>(nb, n));
    const std::vector<int64_t> *bnd = nullptr;
    if (bounds && !exact) {  // explicit block starts (nb + 1, from 0 to n, nondecreasing)
        if (bounds->size() < 2 || bounds->front() != 0 || bounds->back() != n)
            throw Error("PCILU: block bounds must run from 0 to n");
        for (size_t k = 0; k + 1 < bounds->size(); ++k)
            if ((*bounds)[k + 1] <= (*bounds)[k]) throw Error("PCILU: empty or decreasing block");
        bstart_h = *bounds;
        nblocks = (int64_t)bounds->size() - 1;
        bstart.alloc(bstart_h.size());
        HIPCHK(hipMemcpyAsync(bstart.p, bstart_h.data(), sizeof(int64_t) * bstart_h.size(), hipMemcpyHostToDevice, c.st));
        bnd = &bstart_h;
    }
    WindowSpec w{};
    if (nblocks > 1) {
        w.mode = 1;
        w.nblocks = nblocks;
        w.bstart = bnd ? bstart.p : nullptr;
    } else {
        w.mode = 0;
        w.c0 = 0;
        w.c1 = M.halo ? n : M.ncols;  // distributed: drop ghost columns (rank block only)
    }
    if (exact) envelope_csr(M, F, c);
    else extract_csr(M, 0, n, w, 0, n, F, c);
    if (F.max_row > ilu0_max_row()) throw Error("ILU(0): row too long for the LDS-staged factorization");
    diag.alloc(std::max<int64_t>(n, 1));
    dinv.alloc(std::max<int64_t>(n, 1));
    DBuf<int32_t> fail(1);
    HIPCHK(hipMemsetAsync(fail.p, 0, sizeof(int32_t), c.st));
    launch_find_diag(n, F.rp.p, F.ci.p, diag.p, fail.p, c.st);
    std::vector<int64_t> rp(n + 1), dg(n);
    std::vector<int32_t> ci(F.nnz);
    HIPCHK(hipMemcpyAsync(rp.data(), F.rp.p, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, c.st));
    if (F.nnz) HIPCHK(hipMemcpyAsync(ci.data(), F.ci.p, sizeof(int32_t) * F.nnz, hipMemcpyDeviceToHost, c.st));
    int32_t hfail = 0;
    HIPCHK(hipMemcpyAsync(&hfail, fail.p, sizeof(int32_t), hipMemcpyDeviceToHost, c.st));
    c.sync();
    if (hfail) throw Error("ILU(0): missing diagonal entry (PETSc: MAT_FACTOR_STRUCT_ZEROPIVOT)");
    HIPCHK(hipMemcpyAsync(dg.data(), diag.p, sizeof(int64_t) * n, hipMemcpyDeviceToHost, c.st));
    c.sync();
    // numeric factorization, level by level (global levels of the forward sweep)
    mark("extract + download");
    std::vector<int32_t> ordL;
    std::vector<int64_t> Lptr;
    nlev_L = level_order(n, rp, ci, false, ordL, Lptr);
    mark("level order");
    if (sgs) {
        launch_sgs_factor(n, F.rp.p, F.ci.p, F.val.p, diag.p, dinv.p, fail.p, c.st);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(&hfail, fail.p, sizeof(int32_t), hipMemcpyDeviceToHost, c.st));
        c.sync();
    } else {
        // LDS sizing: the most staged entries one row needs
        int64_t max_staged = 0;
        {
            const int T = (int)std::max<int64_t>(1, std::min<int64_t>(16, n / 65536));
            std::vector<int64_t> ms(T, 0);
            std::vector<std::thread> th;
            for (int w = 0; w < T; ++w)
                th.emplace_back([&, w] {
                    for (int64_t i = n * w / T; i < n * (w + 1) / T; ++i) {
                        int64_t tot = 0;
                        for (int64_t k = rp[i]; k < dg[i]; ++k) tot += rp[ci[k] + 1] - dg[ci[k]] - 1;
                        ms[w] = std::max(ms[w], tot);
                    }
                });
            for (auto &x : th) x.join();
            for (int w = 0; w < T; ++w) max_staged = std::max(max_staged, ms[w]);
        }
        DBuf<int32_t> rowsL(std::max<int64_t>(n, 1));
        HIPCHK(hipMemcpyAsync(rowsL.p, ordL.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c.st));
        set_ilu0_test_caps(c.ilu0_stage_cap, c.ilu_dep_grid);  // (process-wide: set per factorization)
        // one launch where levels are narrow (FE blocks: ~30 rows per level); wide levels
        // (BJACOBI on the headline: thousands of rows per level) keep a launch per level,
        // which there costs less than the per-row flags (setup 1.42 vs 1.73 s at N = 59)
        const bool dep = c.ilu_factor_dep == 1 ? nlev_L > 1 && n / nlev_L <= 2048 : c.ilu_factor_dep == 2;
        if (dep) {  // one launch; rows wait on their pivot rows' flags
            // the launch is deadlock-free only if the draw order is a topological
            // order of the pivot DAG (every pivot row r < i with l_ir != 0 drawn
            // before row i): the lowest unfinished drawn row then always has its
            // pivots done.  level_order gives one by construction; checked here
            // (O(nnz)) so that a wrong order is an error, not a bounded wait
            std::vector<int32_t> pos(n);
            for (int64_t q = 0; q < n; ++q) pos[ordL[q]] = (int32_t)q;
            for (int64_t i = 0; i < n; ++i)
                for (int64_t k = rp[i]; k < dg[i]; ++k)
                    if (pos[ci[k]] >= pos[i])
                        throw Error("ILU(0): factorization draw order is not topological (row " +
                                    std::to_string(i) + " before its pivot row " + std::to_string(ci[k]) + ")");
            DBuf<int32_t> done(std::max<int64_t>(n, 1)), ctr(2);
            launch_ilu0_dep(n, rowsL.p, F.rp.p, F.ci.p, F.val.p, diag.p, dinv.p, fail.p, F.max_row, max_staged,
                            done.p, ctr.p, c.st);
            HIPCHK(hipGetLastError());
            c.sync();  // (done / ctr freed below)
        } else {
            for (int64_t l = 0; l < nlev_L; ++l)
                launch_ilu0_level(Lptr[l + 1] - Lptr[l], rowsL.p + Lptr[l], F.rp.p, F.ci.p, F.val.p, diag.p, dinv.p,
                                  fail.p, F.max_row, max_staged, c.st);
        }
        HIPCHK(hipGetLastError());
        set_ilu0_test_caps(-1, 0);  // (launches above are enqueued with their plan: knobs off for other users)
        HIPCHK(hipMemcpyAsync(&hfail, fail.p, sizeof(int32_t), hipMemcpyDeviceToHost, c.st));
        c.sync();
    }
    if (hfail == 3) throw Error("ILU(0): dependency wait exceeded its bound (set pls.ilu_factor_dep 0)");
    if (hfail) throw Error("ILU(0): zero pivot (PETSc: MAT_FACTOR_NUMERIC_ZEROPIVOT)");
    int64_t blen = n / nblocks + 1;
    if (bnd)
        for (size_t k = 0; k + 1 < bnd->size(); ++k) blen = std::max<int64_t>(blen, (*bnd)[k + 1] - (*bnd)[k]);
    max_len = blen;
    const bool fits_lds = blen <= ilu_lds_max_rows() && gmem_mode != 1;
    // Blocks too long for LDS: one workgroup per block with y itself as the
    // block solution when levels are narrow -- FE blocks in a bandwidth-
    // reducing order have ~30-150 rows per level and ~1,400 levels at 3-D
    // N=12, where one launch per level is launch-latency bound (measured
    // ~19 us per level).  Wide levels keep the grid-wide launch per level.
    const bool narrow = nlev_L > 0 && n / nlev_L <= 2048;
    const bool gmem = allow_lds && !fits_lds && gmem_mode >= 0 && blen <= ilu_gmem_max_rows() &&
                      (narrow || nblocks >= 64 || gmem_mode == 1);
    if (nblocks >= 64 || (fits_lds && allow_lds) || gmem) {
        std::vector<int32_t> oL, oU;
        std::vector<int64_t> gL, gU, fL, fU;
        mark("factor");
        block_level_groups(n, nblocks, rp, ci, false, oL, gL, fL, bnd);
        block_level_groups(n, nblocks, rp, ci, true, oU, gU, fU, bnd);
        mark("block level groups");
        block_levels_h.resize(nblocks);
        for (int64_t b = 0; b < nblocks; ++b) block_levels_h[b] = (fL[b + 1] - fL[b]) + (fU[b + 1] - fU[b]);
        block_start_h = block_starts(n, nblocks, bnd);
        build_tri_sell(*this, rp, dg, oL, gL, &fL, false, Lf, c);
        build_tri_sell(*this, rp, dg, oU, gU, &fU, true, Uf, c);
        mark("tri sell");
        nlev_U = (int64_t)gU.size() - 1;
        use_lds = (allow_lds && fits_lds) || gmem;
        lds_gmem = gmem;
        // the super-window sweep: y-resident blocks (pls.sweep_swin; default where
        // the ring sweep would run)
        if (gmem && c.sweep_swin != 0 && (c.sweep_swin == 1 || ring_mode != 0)) {
            const std::vector<int64_t> bst = block_starts(n, nblocks, bnd);
            std::vector<double> fv(F.nnz);
            if (F.nnz) HIPCHK(hipMemcpyAsync(fv.data(), F.val.p, sizeof(double) * F.nnz, hipMemcpyDeviceToHost, c.st));
            c.sync();
            build_swin_tri(nblocks, bst, rp, ci, dg, fv, false, Lsw, c);
            build_swin_tri(nblocks, bst, rp, ci, dg, fv, true, Usw, c);
            std::vector<int64_t> wf(nblocks + 1, 0);
            for (int64_t b = 0; b < nblocks; ++b) wf[b + 1] = wf[b] + (bst[b + 1] - bst[b] + 63) / 64;
            wstart.alloc(nblocks + 1);
            HIPCHK(hipMemcpyAsync(wstart.p, wf.data(), sizeof(int64_t) * (nblocks + 1), hipMemcpyHostToDevice, c.st));
            c.sync();
            swin = true;
            mark("super-window tables");
        }
        auto build_windows = [&](const std::vector<int64_t> &bst) {
            window_max_entries_lu(nblocks, bst, rp, ci, dg, window_entries_L, window_entries_U);
            if (c.window_kpw == 8) window_entries_L = window_entries_U = 32;
            window_entries = std::max(window_entries_L, window_entries_U);
            std::vector<double> fv(F.nnz);
            if (F.nnz) HIPCHK(hipMemcpyAsync(fv.data(), F.val.p, sizeof(double) * F.nnz, hipMemcpyDeviceToHost, c.st));
            c.sync();
            build_window_tri(nblocks, bst, rp, ci, dg, fv, false, Lw, c);
            build_window_tri(nblocks, bst, rp, ci, dg, fv, true, Uw, c);
            mark("window triangles");
            std::vector<int64_t> wf(nblocks + 1, 0);
            for (int64_t b = 0; b < nblocks; ++b) wf[b + 1] = wf[b] + (bst[b + 1] - bst[b] + 63) / 64;
            wstart.alloc(nblocks + 1);
            HIPCHK(hipMemcpyAsync(wstart.p, wf.data(), sizeof(int64_t) * (nblocks + 1), hipMemcpyHostToDevice, c.st));
            c.sync();
        };
        const int64_t lev = (int64_t)gL.size() - 1 + (int64_t)gU.size() - 1;
        auto window_count = [&](const std::vector<int64_t> &bst) {
            int64_t nwin = 0;
            for (int64_t b = 0; b < nblocks; ++b) nwin += 2 * ((bst[b + 1] - bst[b] + 63) / 64);
            return nwin;
        };
        auto ring_fits = [&] {
            return c.window_ring != 0 && blen <= ilu_window_ring_max_rows() &&
                   window_max_reach(n, rp, ci) <= ilu_window_ring_rows() - 64;
        };
        // the window sweep's ring variant on blocks too long for LDS (the classical
        // AMG's np=8 hybrid Gauss-Seidel chunks beyond 19,904 rows: swelling N=160,
        // footing N=80), optionally with the L triangle by levels (the y-resident
        // workgroup sweep; pls.window_mixed).  Cost model, a level ~ a window
        // (measured ~2.4 and ~1.9 us on those chunks): both triangles by levels (the
        // ring sweep) levL + levU, both by windows 2 nw, mixed levL + nw; windows
        // where they save a fifth.  Swelling N=160 (per chunk): L 110 levels, U 666,
        // 403 windows per triangle -- mixed; footing N=80: L 154, U 1,034, 467.
        if (gmem && !swin && c.sweep_window != 0 && ring_fits()) {
            const std::vector<int64_t> bst = block_starts(n, nblocks, bnd);
            const int64_t nw = window_count(bst) / 2, levL = (int64_t)gL.size() - 1;
            const int64_t cost_lev = lev, cost_win = 2 * nw, cost_mix = levL + nw;
            const bool mix = c.window_mixed == 1 || (c.window_mixed == -1 && cost_mix < cost_win);
            // (pls.ilu_gmem 1 -- the y-resident workgroup sweep forced on blocks that fit
            // LDS -- keeps that sweep unless the window sweep is forced too)
            if ((c.sweep_window == 1 || (gmem_mode != 1 && 5 * (mix ? cost_mix : cost_win) <= 4 * cost_lev)) &&
                window_max_entries(nblocks, bst, rp, ci, dg) <= ilu_window_max_entries()) {
                build_windows(bst);
                window = window_ring = true;
                if (mix) {
                    build_lds_tri(*this, n, nblocks, force_lpr, 16, rp, dg, oL, gL, fL, false, Ls, c, nullptr, nullptr,
                                  nullptr, &block_maxsl_h);
                    int64_t wmax = 1;
                    for (size_t k = 0; k + 1 < gL.size(); ++k) wmax = std::max<int64_t>(wmax, gL[k + 1] - gL[k]);
                    std::vector<int32_t> hl(nblocks);
                    HIPCHK(hipMemcpyAsync(hl.data(), Ls.lpr.p, sizeof(int32_t) * nblocks, hipMemcpyDeviceToHost, c.st));
                    c.sync();
                    int lmax = 1;
                    for (int64_t b = 0; b < nblocks; ++b) lmax = std::max(lmax, hl[b]);
                    const int64_t slices = (wmax * lmax + 63) / 64;
                    lds_tpb = slices <= 1 ? 64 : slices <= 4 ? 256 : 1024;
                    zgoff.alloc(nblocks + 1);
                    HIPCHK(hipMemsetAsync(zgoff.p, 0, sizeof(int64_t) * (nblocks + 1), c.st));
                    window_mixed = true;
                }
            }
        }
        // the ring sweep: y-resident blocks whose every level fits one chunk
        if (gmem && ring_mode != 0 && !swin && !window) {
            int64_t wmax = 0;
            for (const auto *g : {&gL, &gU})
                for (size_t k = 0; k + 1 < g->size(); ++k) wmax = std::max<int64_t>(wmax, (*g)[k + 1] - (*g)[k]);
            ring = wmax <= ilu_ring_chunk();
        }
        if (use_lds && !gmem && (c.sweep_chain != 0 || c.sweep_window == 1) && force_lpr == 0) {
            // the chain sweep (one wave per block, 16-lane steps in order, up to 32
            // steps of factor data in flight) for deep, narrow level DAGs: measured
            // ~0.77 us per level for the workgroup sweep on the footing smoother
            // chunks; a chain step costs a fraction of that, so chain when steps <=
            // 3.5 x levels (both triangles)
            const std::vector<int64_t> bst = block_starts(n, nblocks, bnd);
            const std::vector<double> none;
            const int64_t sL = build_chain_tri(nblocks, bst, rp, ci, dg, none, none, oL, gL, fL, false, nullptr, c);
            const int64_t sU = sL < 0 ? -1 : build_chain_tri(nblocks, bst, rp, ci, dg, none, none, oU, gU, fU, true, nullptr, c);
            mark("chain plan");
            const bool deep = sL >= 0 && sU >= 0 && 2 * (sL + sU) <= 7 * lev;
            chain = c.sweep_chain != 0 && sL >= 0 && sU >= 0 && (c.sweep_chain == 1 || deep);
            // the window sweep where the chain would run (or forced): a block's
            // dependent chain becomes its len / 64 windows.  Also where the levels
            // outnumber the windows 2:1 (<= 32 rows per level): the classical AMG's
            // level-0 hybrid Gauss-Seidel chunks under mpirun -np 8 semantics
            // (swelling N=80: 8 chunks of 6,481 rows, ~700 levels per chunk over both
            // triangles) took 790 us per sweep in the workgroup sweep (~1.1 us per
            // level), 745 us in the chain sweep, ~250 us in the window sweep (~1.2 us
            // per window)
            const bool many_levels = lev >= 2 * window_count(bst);
            window = (c.sweep_window == 1 || (c.sweep_window == -1 && c.sweep_chain != 1 && (deep || many_levels))) &&
                     blen <= ilu_window_max_rows() &&
                     window_max_entries(nblocks, bst, rp, ci, dg) <= ilu_window_max_entries();
            if (window) {
                chain = false;
                build_windows(bst);
                window_ring = c.window_ring == 1 && ring_fits();  // (forced: tests compare it with the LDS variant)
            }
            if (chain) {
                std::vector<double> fv(F.nnz), dv(n);
                if (F.nnz) HIPCHK(hipMemcpyAsync(fv.data(), F.val.p, sizeof(double) * F.nnz, hipMemcpyDeviceToHost, c.st));
                if (n) HIPCHK(hipMemcpyAsync(dv.data(), dinv.p, sizeof(double) * n, hipMemcpyDeviceToHost, c.st));
                c.sync();
                build_chain_tri(nblocks, bst, rp, ci, dg, fv, dv, oL, gL, fL, false, &Lc, c);
                build_chain_tri(nblocks, bst, rp, ci, dg, fv, dv, oU, gU, fU, true, &Uc, c);
            }
        }
        if (use_lds && !chain && !window && !swin) {
            const int max_lpr = gmem ? (ring ? 32 : 16) : 4;
            std::vector<int32_t> pL, pU, loL, loU, nlL, nlU;
            if (ring) {
                // rows of a level longest first (slices then take fewer lanes per row
                // as rows get shorter); positions follow this order
                auto sort_levels = [&](std::vector<int32_t> &o, const std::vector<int64_t> &g, bool up) {
                    auto len = [&](int32_t i) { return up ? rp[i + 1] - dg[i] - 1 : dg[i] - rp[i]; };
                    for (size_t k = 0; k + 1 < g.size(); ++k)
                        std::stable_sort(o.begin() + g[k], o.begin() + g[k + 1],
                                         [&](int32_t a, int32_t b) { return len(a) > len(b); });
                };
                sort_levels(oL, gL, false);
                sort_levels(oU, gU, true);
                std::vector<double> fv(F.nnz);
                if (F.nnz) HIPCHK(hipMemcpyAsync(fv.data(), F.val.p, sizeof(double) * F.nnz, hipMemcpyDeviceToHost, c.st));
                c.sync();
                ring_tables(n, nblocks, oL, gL, fL, rp, ci, dg, fv, false, pL, loL, nlL, Lr, c, bnd);
                ring_tables(n, nblocks, oU, gU, fU, rp, ci, dg, fv, true, pU, loU, nlU, Ur, c, bnd);
                // mapUL[b0 + t] = b0 + (L position of the row at U position t)
                std::vector<int32_t> m(n);
                const std::vector<int64_t> bst = block_starts(n, nblocks, bnd);
                int64_t b0 = 0;
                for (int64_t b = 0; b < nblocks; ++b) {
                    const int64_t len = bst[b + 1] - bst[b];
                    for (int64_t t = b0; t < b0 + len; ++t) m[t] = (int32_t)(b0 + pL[oU[t]]);
                    b0 += len;
                }
                mapUL.alloc(std::max<int64_t>(n, 1));
                HIPCHK(hipMemcpyAsync(mapUL.p, m.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c.st));
                c.sync();
            }
            build_lds_tri(*this, n, nblocks, force_lpr, max_lpr, rp, dg, oL, gL, fL, false, Ls, c, ring ? &pL : nullptr,
                          ring ? &loL : nullptr, ring ? &nlL : nullptr, &block_maxsl_h);
            build_lds_tri(*this, n, nblocks, force_lpr, max_lpr, rp, dg, oU, gU, fU, true, Us, c, ring ? &pU : nullptr,
                          ring ? &loU : nullptr, ring ? &nlU : nullptr, &block_maxsl_h);
            // threads per workgroup: as few waves as the widest level's slices need
            // (narrow, deep levels -- FE rows in their natural order, nearly one
            // level per row -- pay a workgroup barrier per level: 16 waves cost
            // ~0.6 us per level, one wave far less).  pls.sweep_tpb overrides.
            int64_t wmax = 1;
            for (const auto *g : {&gL, &gU})
                for (size_t k = 0; k + 1 < g->size(); ++k) wmax = std::max<int64_t>(wmax, (*g)[k + 1] - (*g)[k]);
            int lmax = 1;
            {
                std::vector<int32_t> hl(nblocks), hu(nblocks);
                HIPCHK(hipMemcpyAsync(hl.data(), Ls.lpr.p, sizeof(int32_t) * nblocks, hipMemcpyDeviceToHost, c.st));
                HIPCHK(hipMemcpyAsync(hu.data(), Us.lpr.p, sizeof(int32_t) * nblocks, hipMemcpyDeviceToHost, c.st));
                c.sync();
                for (int64_t b = 0; b < nblocks; ++b) lmax = std::max(lmax, std::max(hl[b], hu[b]));
            }
            const int64_t slices = (wmax * lmax + 63) / 64;
            lds_tpb = slices <= 1 ? 64 : slices <= 4 ? 256 : 1024;
            // (the round-robin level sweep, pls.sweep_rr 1, is bitwise the same and was
            // measured slower on the footing N=128 smoother chunks: 0.83 vs 0.77 us per
            // level -- the per-level cost there is not memory latency)
        }
    } else {
        std::vector<int32_t> ordU;
        std::vector<int64_t> Uptr;
        nlev_U = level_order(n, rp, ci, true, ordU, Uptr);
        if (gmem_mode == -2 && !exact) {
            csr_levels = true;
            lrowsL.alloc(std::max<int64_t>(n, 1));
            lrowsU.alloc(std::max<int64_t>(n, 1));
            HIPCHK(hipMemcpyAsync(lrowsL.p, ordL.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c.st));
            HIPCHK(hipMemcpyAsync(lrowsU.p, ordU.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c.st));
            lptrL = Lptr;
            lptrU = Uptr;
            c.sync();
        } else {
            build_tri_sell(*this, rp, dg, ordL, Lptr, nullptr, false, Lf, c);
            build_tri_sell(*this, rp, dg, ordU, Uptr, nullptr, true, Uf, c);
        }
    }
    if (c.ilu_view)
        fprintf(stderr, "[pls ilu] type %s n %lld blocks %lld max_len %lld levels %lld/%lld sweep %s%s\n", type.c_str(),
                (long long)n, (long long)nblocks, (long long)max_len, (long long)nlev_L, (long long)nlev_U,
                sweep_kind(),
                window ? (" (records " + std::to_string(window_records(window_entries_L)) + "/" +
                          std::to_string(window_records(window_entries_U)) + ")").c_str()
                       : "");
}

void PCILU::apply_blocks(const double *x, double *y, Ctx &c, int64_t b_lo, int64_t b_hi, int rr_group, int tpb,
                         int depth, int64_t *prof) {
    if (!can_apply_blocks()) throw Error("PCILU: block subsets need the LDS sweep");
    const int rr = rr_group > 0 ? rr_group : (lds_rr ? 1 : 0);
    launch_ilu_blocks_lds(n, nblocks, Lf.goff.p, Ls.gslice.p, Ls.sptr.p, Ls.col.p, Ls.val.p, Ls.lpr.p, Uf.goff.p,
                          Us.gslice.p, Us.sptr.p, Us.col.p, Us.val.p, Us.lpr.p, x, y, c.st, prof, false,
                          tpb > 0 ? tpb : lds_tpb, rr, bstart_h.empty() ? nullptr : bstart.p, max_len, b_lo, b_hi,
                          depth == 2 ? lds_depth : depth);
}

const char *PCILU::sweep_kind() const {
    if (!use_lds) return csr_levels ? "levels-csr" : "levels";
    if (swin) return "swin";
    if (ring) return "ring";
    if (window) return window_mixed ? "levels+window-ring" : window_ring ? "window-ring" : "window";
    if (chain) return "chain";
    return lds_gmem ? "gmem" : "lds";
}

void PCILU::apply(const double *x, double *y, Ctx &c) {
    if (use_lds && swin) {
        launch_ilu_blocks_swin(n, nblocks, bstart_h.empty() ? nullptr : bstart.p, wstart.p, Lsw.bsw.p, Lsw.sw.p,
                               Lsw.wnear.p, Lsw.ncol.p, Lsw.nval.p, Lsw.wfar.p, Lsw.fcol.p, Lsw.fval.p, Lsw.tinv.p,
                               Usw.bsw.p, Usw.sw.p, Usw.wnear.p, Usw.ncol.p, Usw.nval.p, Usw.wfar.p, Usw.fcol.p,
                               Usw.fval.p, Usw.tinv.p, x, y, std::max(Lsw.lds_bytes, Usw.lds_bytes), c.st);
        return;
    }
    if (use_lds && ring) {
        auto &sc = ring_scratch[c.st];  // per stream: the concurrent 3-way sweeps share this PC
        if (sc.first.n < (size_t)n) {
            sc.first.alloc(std::max<int64_t>(n, 1));
            sc.second.alloc(std::max<int64_t>(n, 1));
        }
        launch_ilu_blocks_ring(n, nblocks, Lf.goff.p, Ls.gslice.p, Ls.sptr.p, Ls.col.p, Ls.val.p, Ls.lpr.p, Uf.goff.p,
                               Us.gslice.p, Us.sptr.p, Us.col.p, Us.val.p, Us.lpr.p, Lr.coff.p, Lr.cg.p, Lr.cp.p,
                               Ur.coff.p, Ur.cg.p, Ur.cp.p, Lr.ord.p, mapUL.p, Ur.ord.p, Lr.frp.p, Lr.fcol.p,
                               Lr.fval.p, Ur.frp.p, Ur.fcol.p, Ur.fval.p, x, y, sc.first.p, sc.second.p, c.st,
                               lds_tpb, bstart_h.empty() ? nullptr : bstart.p);
        return;
    }
    if (use_lds && window && window_mixed) {  // L: the y-resident level sweep; U: the ring windows
        launch_ilu_blocks_lds(n, nblocks, Lf.goff.p, Ls.gslice.p, Ls.sptr.p, Ls.col.p, Ls.val.p, Ls.lpr.p, zgoff.p,
                              Ls.gslice.p, Ls.sptr.p, Ls.col.p, Ls.val.p, Ls.lpr.p, x, y, c.st, nullptr, true, lds_tpb,
                              0, bstart_h.empty() ? nullptr : bstart.p, max_len, -1, -1, 2);
        launch_ilu_blocks_window(n, nblocks, bstart_h.empty() ? nullptr : bstart.p, wstart.p, Lw.woff.p, Lw.rec.p,
                                 Lw.tinv.p, Uw.woff.p, Uw.rec.p, Uw.tinv.p, y, y, max_len, c.st,
                                 c.window_depth, true, 2, window_entries_L, window_entries_U);
        return;
    }
    if (use_lds && window) {
        launch_ilu_blocks_window(n, nblocks, bstart_h.empty() ? nullptr : bstart.p, wstart.p, Lw.woff.p, Lw.rec.p,
                                 Lw.tinv.p, Uw.woff.p, Uw.rec.p, Uw.tinv.p, x, y, max_len, c.st,
                                 c.window_depth, window_ring, 3, window_entries_L, window_entries_U);
        return;
    }
    if (use_lds && chain) {
        launch_ilu_blocks_chain(n, nblocks, bstart_h.empty() ? nullptr : bstart.p, Lc.base.p, Lc.soff.p, Lc.sz.p,
                                Lc.nsl.p, Lc.lpr.p, Lc.col.p, Lc.val.p, Uc.base.p, Uc.soff.p, Uc.sz.p, Uc.nsl.p,
                                Uc.lpr.p, Uc.col.p, Uc.val.p, x, y, max_len, c.st);
        return;
    }
    if (use_lds) {
        DBuf<int64_t> prof;
        if (!profile_tag.empty()) prof.alloc(nblocks * 8);
        launch_ilu_blocks_lds(n, nblocks, Lf.goff.p, Ls.gslice.p, Ls.sptr.p, Ls.col.p, Ls.val.p, Ls.lpr.p, Uf.goff.p,
                              Us.gslice.p, Us.sptr.p, Us.col.p, Us.val.p, Us.lpr.p, x, y, c.st, prof.p, lds_gmem,
                              lds_tpb, lds_rr ? 1 : 0, bstart_h.empty() ? nullptr : bstart.p, max_len, -1, -1,
                              lds_gmem ? 2 : lds_depth);
        if (!profile_tag.empty()) {
            // diagnostics: per-block sweep times (100 MHz wall clock), slowest first
            std::vector<int64_t> h(nblocks * 8);
            HIPCHK(hipMemcpyAsync(h.data(), prof.p, sizeof(int64_t) * h.size(), hipMemcpyDeviceToHost, c.st));
            c.sync();
            int64_t tmin = INT64_MAX, tmax = 0;
            std::vector<int64_t> order(nblocks);
            for (int64_t b = 0; b < nblocks; ++b) {
                order[b] = b;
                tmin = std::min(tmin, h[b * 8]);
                tmax = std::max(tmax, h[b * 8 + 2]);
            }
            std::sort(order.begin(), order.end(),
                      [&](int64_t a, int64_t b) { return h[a * 8 + 2] - h[a * 8] > h[b * 8 + 2] - h[b * 8]; });
            fprintf(stderr, "[sweep %s] %lld blocks, kernel span %.1f us\n", profile_tag.c_str(), (long long)nblocks,
                    (tmax - tmin) * 0.01);
            for (int64_t r = 0; r < std::min<int64_t>(nblocks, 12); ++r) {
                const int64_t b = order[r], *p = &h[b * 8];
                fprintf(stderr,
                        "  blk %4lld rows %6lld start %+8.1f us  L %7.1f us (%4lld lv, %5lld sl)  U %7.1f us (%4lld lv)"
                        "  lanes/row L,U %lld,%lld\n",
                        (long long)b, (long long)p[5], (p[0] - tmin) * 0.01, (p[1] - p[0]) * 0.01, (long long)p[3],
                        (long long)p[6], (p[2] - p[1]) * 0.01, (long long)p[4], (long long)(p[7] / 10),
                        (long long)(p[7] % 10));
            }
            profile_tag.clear();
        }
        return;
    }
    if (csr_levels) {
        for (int64_t l = 0; l < nlev_L; ++l)
            launch_tri_csr_level(lptrL[l + 1] - lptrL[l], lrowsL.p + lptrL[l], F.rp.p, F.ci.p, F.val.p, diag.p,
                                 dinv.p, 0, x, y, c.st);
        for (int64_t l = 0; l < nlev_U; ++l)
            launch_tri_csr_level(lptrU[l + 1] - lptrU[l], lrowsU.p + lptrU[l], F.rp.p, F.ci.p, F.val.p, diag.p,
                                 dinv.p, 1, y, y, c.st);
        return;
    }
    Lf.apply(x, y, c);
    Uf.apply(y, y, c);
}

PCDenseLU::PCDenseLU(const DevCSR &M, Ctx &c, double u) {
    type = "lu";
    n = M.nrows;
    if (M.ncols != n) throw Error("lu: block is not square");
    ld = std::max<int64_t>(64, (n + 63) / 64 * 64);
    inv.alloc(ld * ld);
    launch_dense_from_csr(n, ld, M.rp.p, M.ci.p, M.val.p, inv.p, c.st);
    DBuf<double> D(64 * 64), P;
    DBuf<int32_t> fail(1), st;
    HIPCHK(hipMemsetAsync(fail.p, 0, sizeof(int32_t), c.st));
    if (u > 0.0 && n > 1) {  // MUMPS-style threshold partial pivoting over every remaining row
        std::vector<int32_t> id(n);
        std::iota(id.begin(), id.end(), 0);
        rowperm.alloc(n);
        HIPCHK(hipMemcpyAsync(rowperm.p, id.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c.st));
        P.alloc((size_t)n * 64 + panel_fast_doubles());
        st.alloc(3);
        HIPCHK(hipMemsetAsync(st.p, 0, sizeof(int32_t) * 3, c.st));
        c.sync();  // (id)
    }
    launch_dense_invert(ld, inv.p, D.p, fail.p, c.st, n, P.p, rowperm.p, st.p, rowperm.p ? u : 0.0);
    HIPCHK(hipGetLastError());
    int32_t hfail = 0;
    HIPCHK(hipMemcpyAsync(&hfail, fail.p, sizeof(int32_t), hipMemcpyDeviceToHost, c.st));
    if (st.p) HIPCHK(hipMemcpyAsync(piv_stats, st.p, sizeof(int32_t) * 3, hipMemcpyDeviceToHost, c.st));
    c.sync();
    if (hfail) throw Error("LU: zero pivot (PETSc: MAT_FACTOR_NUMERIC_ZEROPIVOT)");
}

void PCDenseLU::apply(const double *x, double *y, Ctx &c) {
    launch_dense_gemv(n, ld, inv.p, x, y, c.st, rowperm.p);
}

void csr_bandwidths(const DevCSR &M, int64_t &kl, int64_t &ku, Ctx &c) {
    const int64_t n = M.nrows;
    kl = ku = 0;
    if (n == 0) return;
    std::vector<int64_t> rp(n + 1);
    std::vector<int32_t> ci(M.nnz);
    HIPCHK(hipMemcpyAsync(rp.data(), M.rp.p, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, c.st));
    if (M.nnz) HIPCHK(hipMemcpyAsync(ci.data(), M.ci.p, sizeof(int32_t) * M.nnz, hipMemcpyDeviceToHost, c.st));
    c.sync();
    for (int64_t i = 0; i < n; ++i) {
        if (rp[i + 1] == rp[i]) continue;
        kl = std::max<int64_t>(kl, i - ci[rp[i]]);
        ku = std::max<int64_t>(ku, ci[rp[i + 1] - 1] - i);
    }
}

PCBandLU::PCBandLU(const DevCSR &M, int64_t kl, int64_t ku, Ctx &c, int64_t spike_plen) {
    type = "lu";
    n = M.nrows;
    if (M.ncols != n) throw Error("lu: block is not square");
    nb = (n + 63) / 64;
    bl = (kl + 63) / 64;
    bu = (ku + 63) / 64;
    const int64_t W = bl + bu + 1;
    T.alloc((size_t)(nb * W) * 4096);
    Dl.alloc((size_t)nb * 4096);
    Du.alloc((size_t)nb * 4096);
    Gl.alloc((size_t)nb * 4096);
    Gu.alloc((size_t)nb * 4096);
    t.alloc(std::max<int64_t>(n, 1));
    G.alloc((size_t)std::max<int64_t>(nb, 1) * 128);
    fail.alloc(1);
    ticket.alloc(1);
    HIPCHK(hipMemsetAsync(G.p, 0, sizeof(uint64_t) * G.n, c.st));
    HIPCHK(hipMemsetAsync(fail.p, 0, sizeof(int32_t), c.st));
    HIPCHK(hipMemsetAsync(ticket.p, 0, sizeof(uint64_t), c.st));
    launch_band_from_csr(n, nb, bl, bu, M.rp.p, M.ci.p, M.val.p, T.p, c.st);
    launch_band_factor(nb, bl, bu, T.p, Dl.p, Du.p, Gl.p, Gu.p, fail.p, c.st);
    HIPCHK(hipGetLastError());
    if (check_fail(c)) throw Error("LU: zero pivot (PETSc: MAT_FACTOR_NUMERIC_ZEROPIVOT)");
    // SPIKE partitions (band.hip): ~16 concurrent chains per triangle (footing
    // N=128 Schur block, 2,064 tile rows: 16 -> 201 it/s, 32 -> 195, 64 -> 194)
    const int64_t bwmax = std::max<int64_t>(std::max(bl, bu), 1);
    int64_t pl = spike_plen < 0 ? std::max(bwmax, (nb + 15) / 16) : spike_plen;
    if (pl > 0) {
        pl = std::max(pl, bwmax);
        pl += pl & 1;  // whole super-rows
    }
    if (pl > 0 && pl < nb && (bl > 0 || bu > 0)) {
        plen = pl;
        spike_tmp.alloc((size_t)std::max<int64_t>(spike_scratch_doubles(bwmax), 1));
        if (bl > 0) {
            Wl.alloc((size_t)(nb * bl) * 4096);
            launch_spike_setup(nb, bl, bu, 0, plen, T.p, Dl.p, Wl.p, c.st);
        }
        if (bu > 0) {
            Wu.alloc((size_t)(nb * bu) * 4096);
            launch_spike_setup(nb, bl, bu, 1, plen, T.p, Du.p, Wu.p, c.st);
        }
        HIPCHK(hipGetLastError());
        c.sync();
    }
}

int32_t PCBandLU::check_fail(Ctx &c) {
    int32_t h = 0;
    HIPCHK(hipMemcpyAsync(&h, fail.p, sizeof(int32_t), hipMemcpyDeviceToHost, c.st));
    c.sync();
    return h;
}

void PCBandLU::apply(const double *x, double *y, Ctx &c) {
    // epochs 2s+1, 2s+2 (never 0); each sweep draws band_sweep_tickets(nb) tickets
    const uint64_t nt = (uint64_t)band_sweep_tickets(nb);
    launch_band_sweep(n, nb, bl, bu, T.p, Dl.p, Gl.p, x, t.p, G.p, ticket.p, sweeps * nt, (uint32_t)(sweeps + 1), 0,
                      fail.p, c.st, plen);
    ++sweeps;
    if (plen > 0 && bl > 0) launch_spike_apply(n, nb, bl, 0, plen, Wl.p, t.p, spike_tmp.p, c.st);
    launch_band_sweep(n, nb, bl, bu, T.p, Du.p, Gu.p, t.p, y, G.p, ticket.p, sweeps * nt, (uint32_t)(sweeps + 1), 1,
                      fail.p, c.st, plen);
    ++sweeps;
    if (plen > 0 && bu > 0) launch_spike_apply(n, nb, bu, 1, plen, Wu.p, y, spike_tmp.p, c.st);
}

std::unique_ptr<PC> make_lu(const DevCSR &M, const Options &o, Ctx &c) {
    const std::string path = o.str("pls.lu_path", "auto");
    if (path != "auto" && path != "dense" && path != "sparse" && path != "band" && path != "envelope")
        throw Error("pls.lu_path " + path + " (auto, dense, sparse, band, envelope)");
    if (path == "dense" || (path == "auto" && M.nrows <= o.integer("pls.lu_dense_max", 32768))) {
        auto pc = std::make_unique<PCDenseLU>(M, c, o.num("pls.lu_pivot_threshold", 0.01));
        if (o.flag("pls.lu_view", false))
            fprintf(stderr, "[dense lu] n %lld: threshold pivoting u = %g: %d rows exchanged, %d pivots below u x "
                    "column max (delayed by MUMPS), %d zero columns\n", (long long)M.nrows,
                    o.num("pls.lu_pivot_threshold", 0.01), pc->piv_stats[0], pc->piv_stats[1], pc->piv_stats[2]);
        return pc;
    }
    // larger blocks: nested dissection + multifrontal LU (the MUMPS stand-in)
    if (path == "sparse" || path == "auto") return make_sparse_lu(M, o, c);
    if (path == "band") {
        int64_t kl = 0, ku = 0;
        csr_bandwidths(M, kl, ku, c);
        // band tiles + the SPIKE spikes (nb x (bl + bu) tiles): ~2x the band.  Default cap:
        // 3/4 of the card's HBM (288 GB per MI355X: the 2-D footing N=128 Schur block's
        // 95 GB band + 95 GB of spikes fit; an allocation that then fails is reported),
        // pls.lu_band_max_gb overrides
        return std::make_unique<PCBandLU>(M, kl, ku, c, o.integer("pls.band_spike_plen", -1));
    }
    // the envelope (profile) LU: exact, level-scheduled
    return std::make_unique<PCILU>(M, 1, c, true, o.flag("pls.ilu_lds", true), 0, (int)o.integer("pls.ilu_gmem", 0),
                                   (int)o.integer("pls.ilu_ring", 1));
}

// Gather a sharded diagonal block -- every rank's MPIAIJ rows with
// block-global columns (Halo::l2g) -- into the global host CSR, in the block's
// global order, on every rank (host allgather, setup only).  srcslot[g]: where
// global row g sits in a padded allgather of the ranks' rows (q * maxloc + i);
// rank_rows: the ranks' row counts when they own contiguous ranges in rank
// order (every single-field block, every caller-assembled one), else empty.
HostCSR gather_block(const DevCSR &M, Ctx &c, const std::string &prefix, std::vector<int64_t> &srcslot,
                     int64_t &maxloc, std::vector<int64_t> &rank_rows) {
    const int64_t nloc = M.nrows;
    const Halo &H = *M.halo;
    if ((int64_t)H.l2g.size() < M.ncols || H.nlocal != M.nrows)
        throw Error("redundant PC (prefix " + prefix + "): block is not a diagonal block of the sharded system");
    Comm &cm = *c.comm;
    const int G = cm.size;
    const HostCSR L = download(M, c);
    std::vector<int64_t> cnt{nloc, (int64_t)L.ci.size()}, all(2 * G);
    cm.allgather_host(cnt.data(), sizeof(int64_t) * 2, all.data());
    int64_t maxnnz = 0, N = 0;
    maxloc = 0;
    for (int q = 0; q < G; ++q) {
        maxloc = std::max(maxloc, all[2 * q]);
        maxnnz = std::max(maxnnz, all[2 * q + 1]);
        N += all[2 * q];
    }
    // message: rows (global ids), row lengths, columns (global), values -- padded to the largest rank's
    const int64_t words = 2 * maxloc + 2 * maxnnz;
    std::vector<int64_t> msg(words, 0), recv((size_t)words * G);
    for (int64_t i = 0; i < nloc; ++i) {
        msg[i] = H.l2g[i];
        msg[maxloc + i] = L.rp[i + 1] - L.rp[i];
    }
    for (size_t k = 0; k < L.ci.size(); ++k) {
        msg[2 * maxloc + k] = H.l2g[L.ci[k]];
        std::memcpy(&msg[2 * maxloc + maxnnz + k], &L.v[k], sizeof(double));
    }
    cm.allgather_host(msg.data(), sizeof(int64_t) * words, recv.data());
    // global CSR: row g from its owner, columns sorted
    std::vector<int64_t> rowlen(N, -1);
    srcslot.assign(N, -1);
    for (int q = 0; q < G; ++q) {
        const int64_t *m = recv.data() + (size_t)words * q;
        for (int64_t i = 0; i < all[2 * q]; ++i) {
            const int64_t g = m[i];
            if (g < 0 || g >= N || rowlen[g] >= 0) throw Error("redundant PC: inconsistent row ownership");
            rowlen[g] = m[maxloc + i];
            srcslot[g] = q * maxloc + i;
        }
    }
    HostCSR Gh;
    Gh.nrows = Gh.ncols = N;
    Gh.rp.assign(N + 1, 0);
    for (int64_t g = 0; g < N; ++g) Gh.rp[g + 1] = Gh.rp[g] + rowlen[g];
    Gh.ci.resize(Gh.rp[N]);
    Gh.v.resize(Gh.rp[N]);
    std::vector<std::pair<int64_t, double>> row;
    for (int q = 0; q < G; ++q) {
        const int64_t *m = recv.data() + (size_t)words * q;
        int64_t k = 0;
        for (int64_t i = 0; i < all[2 * q]; ++i) {
            const int64_t g = m[i], len = m[maxloc + i];
            row.resize(len);
            for (int64_t e = 0; e < len; ++e, ++k) {
                double v;
                std::memcpy(&v, &m[2 * maxloc + maxnnz + k], sizeof(double));
                row[e] = {m[2 * maxloc + k], v};
            }
            std::sort(row.begin(), row.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
            for (int64_t e = 0; e < len; ++e) {
                Gh.ci[Gh.rp[g] + e] = (int32_t)row[e].first;
                Gh.v[Gh.rp[g] + e] = row[e].second;
            }
        }
    }
    rank_rows.clear();
    bool contiguous = true;
    int64_t start = 0;
    for (int q = 0; q < G && contiguous; ++q) {
        const int64_t *m = recv.data() + (size_t)words * q;
        for (int64_t i = 0; i < all[2 * q]; ++i)
            if (m[i] != start + i) contiguous = false;
        start += all[2 * q];
    }
    if (contiguous)
        for (int q = 0; q < G; ++q) rank_rows.push_back(all[2 * q]);
    return Gh;
}

// Local rows L (columns: global indices of a column space owned in contiguous
// rank ranges cst[q] .. cst[q + 1]) -> a distributed DevCSR: owned columns ->
// local [0, nlocal), referenced others -> ghosts nlocal + k in global order
// (= owner-major), the halo plan by one alltoallv of index lists, entries of a
// row sorted by local column, the SpMV layout built.  Every rank calls it.
void upload_dist(const HostCSR &L, const std::vector<int64_t> &cst, DevCSR &M, Ctx &c) {
    Comm &cm = *c.comm;
    const int G = cm.size, r = cm.rank;
    if ((int)cst.size() != G + 1) throw Error("upload_dist: one column range per rank expected");
    const int64_t c0 = cst[r], nlocal = cst[r + 1] - cst[r];
    std::vector<int64_t> gh;
    for (int32_t j : L.ci)
        if (j < c0 || j >= c0 + nlocal) gh.push_back(j);
    std::sort(gh.begin(), gh.end());
    gh.erase(std::unique(gh.begin(), gh.end()), gh.end());
    auto H = std::make_shared<Halo>();
    H->nlocal = nlocal;
    H->nghost = (int64_t)gh.size();
    std::vector<std::vector<int64_t>> need(G), asked;
    H->rcnt.assign(G, 0);
    H->roff.assign(G, 0);
    {
        size_t k = 0;
        for (int q = 0; q < G; ++q) {
            H->roff[q] = (int64_t)k;
            while (k < gh.size() && gh[k] < cst[q + 1]) need[q].push_back(gh[k++]);
            H->rcnt[q] = (int64_t)need[q].size();
        }
    }
    cm.alltoallv_i64(need, asked);
    std::vector<int32_t> sidx;
    H->scnt.assign(G, 0);
    H->soff.assign(G, 0);
    for (int q = 0; q < G; ++q) {
        H->soff[q] = (int64_t)sidx.size();
        for (int64_t g : asked[q]) {
            if (g < c0 || g >= c0 + nlocal) throw Error("halo plan: peer asked for a column this rank does not own");
            sidx.push_back((int32_t)(g - c0));
        }
        H->scnt[q] = (int64_t)asked[q].size();
    }
    H->nsend = (int64_t)sidx.size();
    H->send_idx.alloc(std::max<int64_t>(H->nsend, 1));
    if (H->nsend) HIPCHK(hipMemcpyAsync(H->send_idx.p, sidx.data(), sizeof(int32_t) * H->nsend, hipMemcpyHostToDevice, c.st));
    H->sendbuf.alloc(std::max<int64_t>(H->nsend, 1));
    H->ghost.alloc(std::max<int64_t>(H->nghost, 1));
    H->l2g.resize(nlocal + gh.size());
    for (int64_t i = 0; i < nlocal; ++i) H->l2g[i] = c0 + i;
    for (size_t k = 0; k < gh.size(); ++k) H->l2g[nlocal + k] = gh[k];
    HostCSR T;
    T.nrows = L.nrows;
    T.ncols = nlocal + (int64_t)gh.size();
    T.rp.assign(1, 0);
    std::vector<std::pair<int32_t, double>> row;
    for (int64_t i = 0; i < L.nrows; ++i) {
        row.clear();
        for (int64_t k = L.rp[i]; k < L.rp[i + 1]; ++k) {
            const int64_t j = L.ci[k];
            const int32_t lj = (j >= c0 && j < c0 + nlocal)
                                   ? (int32_t)(j - c0)
                                   : (int32_t)(nlocal + (std::lower_bound(gh.begin(), gh.end(), j) - gh.begin()));
            row.push_back({lj, L.v[k]});
        }
        std::sort(row.begin(), row.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
        for (auto &e : row) {
            T.ci.push_back(e.first);
            T.v.push_back(e.second);
        }
        T.rp.push_back((int64_t)T.ci.size());
    }
    upload(T, M, c);
    M.ncols = T.ncols;
    M.halo = H;
    M.sell.reset();
    build_sell(M, c);
    c.sync();
}

// a single-rank context carrying c's layout options
std::unique_ptr<Ctx> layout_ctx(const Ctx &c) {
    auto self = std::make_unique<Ctx>();
    self->sell_d16 = c.sell_d16;
    self->d16_wide_lpr = c.d16_wide_lpr;
    self->d16_unroll = c.d16_unroll;
    self->d16_segs = c.d16_segs;
    self->d16_sigma = c.d16_sigma;
    self->d16_sigma_pad = c.d16_sigma_pad;
    self->d16_sorted_lpr = c.d16_sorted_lpr;
    self->spmv_b3 = c.spmv_b3;
    self->spmv_rcm = c.spmv_rcm;
    self->sweep_chain = c.sweep_chain;
    self->sweep_window = c.sweep_window;
    self->window_depth = c.window_depth;
    self->window_ring = c.window_ring;
    self->window_mixed = c.window_mixed;
    self->window_kpw = c.window_kpw;
    self->amg_csr_below = c.amg_csr_below;
    return self;
}

// PETSc PCREDUNDANT semantics for PCs that act on a whole parallel block
// (ILU(0), LU, classical / smoothed-aggregation AMG) when the block is
// sharded over G ranks: every rank gathers the block (its MPIAIJ rows with
// block-global column indices, Halo::l2g) into the global matrix in the
// block's global order, builds the PC on it with a single-rank context, and
// per application allgathers x, applies the PC redundantly and keeps its own
// rows.  The result is the one-rank PC's result on the same block, bitwise.
struct PCRedundant : PC {
    std::unique_ptr<Ctx> self;  // own stream, single-rank communicator
    DevCSR Gm;                  // the gathered global block
    std::unique_ptr<PC> inner;
    int64_t nloc = 0, maxloc = 0, N = 0;
    DBuf<int64_t> src, mine;    // xg[g] = gathered[src[g]];  y[i] = yg[mine[i]]
    DBuf<double> sendbuf, gath, xg, yg;
    hipEvent_t ev_a = nullptr, ev_b = nullptr;

    PCRedundant(const std::string &t, const DevCSR &M, Ctx &c,
                const std::function<std::unique_ptr<PC>(const DevCSR &, Ctx &)> &factory, const std::string &prefix,
                GatheredBlock *pre) {
        type = t;
        n = nloc = M.nrows;
        const Halo &H = *M.halo;
        const int G = c.comm->size;
        GatheredBlock own;
        if (!pre) {
            own.G = gather_block(M, c, prefix, own.srcslot, own.maxloc, own.rank_rows);
            pre = &own;
        }
        const HostCSR &Gh = pre->G;
        const std::vector<int64_t> &srcslot = pre->srcslot, &rank_rows = pre->rank_rows;
        maxloc = pre->maxloc;
        N = Gh.nrows;
        self = layout_ctx(c);
        // the ranks' rows: contiguous ranges in rank order -> the inner PC may restate
        // how the reference's PC runs over G ranks (classical AMG: hypre's per-rank
        // HMIS and smoother)
        self->rank_rows = rank_rows;
        upload(Gh, Gm, *self);
        inner = factory(Gm, *self);
        std::vector<int64_t> mg(H.l2g.begin(), H.l2g.begin() + nloc);
        src.alloc(std::max<int64_t>(N, 1));
        mine.alloc(std::max<int64_t>(nloc, 1));
        HIPCHK(hipMemcpyAsync(src.p, srcslot.data(), sizeof(int64_t) * N, hipMemcpyHostToDevice, c.st));
        if (nloc) HIPCHK(hipMemcpyAsync(mine.p, mg.data(), sizeof(int64_t) * nloc, hipMemcpyHostToDevice, c.st));
        sendbuf.alloc(std::max<int64_t>(maxloc, 1));
        HIPCHK(hipMemsetAsync(sendbuf.p, 0, sizeof(double) * std::max<int64_t>(maxloc, 1), c.st));
        gath.alloc(std::max<int64_t>(maxloc * G, 1));
        xg.alloc(std::max<int64_t>(N, 1));
        yg.alloc(std::max<int64_t>(N, 1));
        HIPCHK(hipEventCreateWithFlags(&ev_a, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev_b, hipEventDisableTiming));
        self->sync();
        c.sync();
    }
    ~PCRedundant() override {
        if (ev_a) (void)hipEventDestroy(ev_a);
        if (ev_b) (void)hipEventDestroy(ev_b);
    }
    void apply(const double *x, double *y, Ctx &c) override {
        if (nloc) launch_copy(nloc, x, sendbuf.p, c.st);
        c.comm->allgather_dev(sendbuf.p, (int)std::max<int64_t>(maxloc, 1), gath.p, c.st);
        launch_gather(N, src.p, gath.p, xg.p, c.st);
        HIPCHK(hipEventRecord(ev_a, c.st));
        HIPCHK(hipStreamWaitEvent(self->st, ev_a, 0));
        inner->apply(xg.p, yg.p, *self);
        HIPCHK(hipEventRecord(ev_b, self->st));
        HIPCHK(hipStreamWaitEvent(c.st, ev_b, 0));
        launch_gather(nloc, mine.p, yg.p, y, c.st);
    }
};

std::unique_ptr<PC> make_redundant(const std::string &type, const DevCSR &M, Ctx &c,
                                   const std::function<std::unique_ptr<PC>(const DevCSR &, Ctx &)> &factory,
                                   const std::string &prefix, GatheredBlock *pre) {
    return std::make_unique<PCRedundant>(type, M, c, factory, prefix, pre);
}

// levels of factor data the LDS sweep keeps in flight: pls.sweep_depth (or
// <prefix>pls_sweep_depth for one PC) 2 (default), 3 or 4 -- bitwise the same sweep
static int sweep_depth_opt(const Options &o, const std::string &prefix) {
    const std::string k = o.has(prefix + "pls_sweep_depth") ? prefix + "pls_sweep_depth" : "pls.sweep_depth";
    const int d = (int)o.integer(k, 2);
    if (d < 2 || d > 4) throw Error(k + " must be 2, 3 or 4");
    return d;
}

std::unique_ptr<PC> make_pc(const std::string &type, const DevCSR &M, const Options &o, const std::string &prefix,
                            Ctx &c) {
    if (type == "none") return std::make_unique<PCNone>(M.nrows);
    if (type == "jacobi") return std::make_unique<PCJacobi>(M, c);
    const bool dist = c.comm && c.comm->size > 1;
    // whole-block PCs on a sharded block: gathered and applied redundantly (PCREDUNDANT)
    if (M.halo && (type == "ilu" || type == "lu" || type == "cholesky" || type == "gamg" || type == "hypre")) {
        // PETSc's own ILU refuses a parallel (MPIAIJ) matrix; MUMPS LU and hypre run
        // distributed.  Redundant ILU is an extension, on request only.
        if (type == "ilu" && !o.flag("pls.redundant_ilu", false))
            throw Error("PC type 'ilu' (prefix " + prefix + ") on a matrix sharded over " +
                        std::to_string(c.comm ? c.comm->size : 1) +
                        " ranks: PETSc's ILU does not run on MPIAIJ matrices (use bjacobi, or pls.redundant_ilu 1 "
                        "for the one-rank ILU applied redundantly)");
        GatheredBlock pre;
        bool gathered = false;
        if (type == "hypre" && o.str("pls.hypre", "boomeramg") == "boomeramg" && o.flag("pls.hypre_dist", true)) {
            // BoomerAMG as under mpirun -np G: the np = G hierarchy, each rank smoothing its
            // own rows (Jacobi across ranks); needs ranks owning contiguous rows in rank order
            pre.G = gather_block(M, c, prefix, pre.srcslot, pre.maxloc, pre.rank_rows);
            gathered = true;
            if (!pre.rank_rows.empty()) return make_boomeramg_dist(M, pre.G, pre.rank_rows, o, prefix, c);
        }
        if (o.flag("pls.redundant_error", false))
            throw Error("PC type '" + type + "' (prefix " + prefix + ") acts on the whole parallel matrix (pls.redundant_error)");
        return make_redundant(type, M, c, [&](const DevCSR &Gm, Ctx &sc) { return make_pc(type, Gm, o, prefix, sc); },
                              prefix, gathered ? &pre : nullptr);
    }
    if (type == "ilu") {
        if (o.integer(prefix + "pc_factor_levels", 0) != 0)
            throw Error(prefix + "pc_factor_levels > 0: only ILU(0) is implemented");
        auto pc = std::make_unique<PCILU>(M, 1, c, false, o.flag("pls.ilu_lds", true), 0,
                                          (int)o.integer("pls.ilu_gmem", 0), (int)o.integer("pls.ilu_ring", 1));
        if (o.has("pls.sweep_tpb")) pc->lds_tpb = (int)o.integer("pls.sweep_tpb", 1024);
        pc->lds_depth = sweep_depth_opt(o, prefix);
        if (o.has("pls.sweep_rr")) pc->lds_rr = o.flag("pls.sweep_rr", false) && pc->use_lds && !pc->ring;
        return pc;
    }
    if (type == "lu" || type == "cholesky") return make_lu(M, o, c);
    if (type == "bjacobi") {
        // total blocks over all ranks (PCBJacobiSetTotalBlocks): rank r gets
        // B / size (+1 for the first B % size ranks); at least one per rank
        const int64_t nbt = o.integer(prefix + "pc_bjacobi_blocks", dist ? c.comm->size : 1);
        int64_t nb = nbt;
        if (dist) nb = std::max<int64_t>(1, nbt / c.comm->size + (c.comm->rank < nbt % c.comm->size ? 1 : 0));
        const std::string sub = o.str(prefix + "sub_pc_type", "ilu");
        if (sub == "ilu") {
            if (o.integer(prefix + "sub_pc_factor_levels", 0) != 0)
                throw Error(prefix + "sub_pc_factor_levels > 0: only ILU(0) is implemented");
            auto pc = std::make_unique<PCILU>(M, nb, c, false, o.flag("pls.ilu_lds", true),
                                              (int)o.integer("pls.sweep_lpr", 0), (int)o.integer("pls.ilu_gmem", 0),
                                              (int)o.integer("pls.ilu_ring", 1));
            if (o.flag("pls.sweep_profile", false)) pc->profile_tag = prefix;
            if (o.has("pls.sweep_tpb")) pc->lds_tpb = (int)o.integer("pls.sweep_tpb", 1024);
            pc->lds_depth = sweep_depth_opt(o, prefix);
            if (o.has("pls.sweep_rr")) pc->lds_rr = o.flag("pls.sweep_rr", false) && pc->use_lds && !pc->ring;
            return pc;
        }
        if (sub == "jacobi") return std::make_unique<PCJacobi>(M, c);
        if (sub == "none") return std::make_unique<PCNone>(M.nrows);
        throw Error(prefix + "sub_pc_type " + sub + " is not available on the device");
    }
    if (type == "gamg") return make_amg(M, o, prefix, false, c);
    if (type == "hypre") {
        // hypre is not in this image: classical AMG restating BoomerAMG as the
        // reference configures it (oracle/boomeramg.py); pls.hypre sa selects
        // the smoothed-aggregation AMG instead, pls.hypre error the refusal
        const std::string h = o.str("pls.hypre", "boomeramg");
        if (h == "error")
            throw Error("PC type 'hypre' (prefix " + prefix + ") is not available (pls.hypre error)");
        if (h == "sa" || h == "gamg") return make_amg(M, o, prefix, true, c);
        if (h != "boomeramg") throw Error("pls.hypre " + h + ": expected boomeramg, sa or error");
        return make_boomeramg(M, o, prefix, c);
    }
    throw Error("PC type '" + type + "' (prefix " + prefix +
                ") is not available in this build (supported: none, jacobi, ilu, bjacobi, lu, gamg, hypre)");
}

// ================================================================= KSP ===
void KSP::resolve_side_norm(const std::string &side, const std::string &nt) {
    // KSPSetUpNorms_Private for the types implemented here
    if (type == "preonly") {
        right = false;
        norm = "none";
        return;
    }
    if (type == "gmres") {
        std::string s = side;
        if (s.empty()) s = (nt == "unpreconditioned") ? "right" : "left";
        std::string nn = nt;
        if (nn.empty()) nn = (s == "right") ? "unpreconditioned" : "preconditioned";
        const bool ok = (s == "left" && (nn == "preconditioned" || nn == "none")) ||
                        (s == "right" && (nn == "unpreconditioned" || nn == "none"));
        if (!ok) throw Error("KSPGMRES (" + prefix + ") does not support norm " + nn + " with pc side " + s);
        right = (s == "right");
        norm = nn;
        return;
    }
    if (type == "cg") {
        if (!side.empty() && side != "left") throw Error("KSPCG (" + prefix + ") supports only left preconditioning");
        right = false;
        norm = nt.empty() ? "preconditioned" : nt;
        if (norm != "preconditioned" && norm != "unpreconditioned" && norm != "none")
            throw Error("KSPCG (" + prefix + "): unsupported norm type " + norm);
        return;
    }
    throw Error("KSP type '" + type + "' (prefix " + prefix + ") is not available (supported: gmres, cg, preonly)");
}

void KSP::ensure_work(Ctx &c) {
    if (type == "gmres") {
        // CGS dots of up to restart + 1 columns: one partial per (column, block)
        // (the context's default room, 136 columns at the largest grid, overflowed
        // past ~450 iterations of a 1.3M-row solve)
        c.ensure_partial(n, restart + 2);
        if (allocated_k != restart) {
            ldv = (n + 63) & ~(int64_t)63;  // 512-B aligned columns (16-B loads)
            V.alloc((size_t)(restart + 1) * ldv);
            t1.alloc(n);
            t2.alloc(n);
            dh.alloc(restart + 4);
            allocated_k = restart;
        }
    } else if (type == "cg") {
        if (allocated_k != 0) {
            t1.alloc(n);  // r
            t2.alloc(n);  // z
            t3.alloc(n);  // p
            t4.alloc(n);  // w
            allocated_k = 0;
        }
    }
}

int KSP::converged(int it, double r) {
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    if (it == 0) {
        rnorm0 = r;
        ttol = std::max(rtol * rnorm0, atol);
        if (time_limit > 0) t_start = now();
    }
    if (std::isnan(r) || std::isinf(r)) return DIVERGED_NANORINF;
    if (r <= ttol) return r < atol ? CONVERGED_ATOL : CONVERGED_RTOL;
    if (r >= dtol * rnorm0) return DIVERGED_DTOL;
    if (time_limit > 0 && it > 0 && now() - t_start > time_limit) return DIVERGED_TIME_LIMIT;
    return CONVERGED_ITERATING;
}

void KSP::solve(const double *b, double *x, Ctx &c) {
    history.clear();
    if (type == "preonly") {
        pc->apply(b, x, c);
        its = 1;
        reason = CONVERGED_ITS;
    } else {
        ensure_work(c);
        if (type == "gmres") solve_gmres(b, x, c);
        else if (type == "cg") {
            // the device-resident loop unless something needs each iteration on the host
            if (cg_device && !monitor && time_limit <= 0 && maxit > 0 && maxit <= 10000000) solve_cg_dev(b, x, c);
            else solve_cg(b, x, c);
        }
        else throw Error("KSP type " + type + " not available");
    }
    stat_its += its;
    stat_max = std::max<int64_t>(stat_max, its);
    ++stat_solves;
    stat_div += reason < 0 ? 1 : 0;
    if (reason < 0) stat_last_neg = reason;
    c.check_bounds();
}

KSP::~KSP() {
    if (stats && stat_solves)
        fprintf(stderr, "[ksp %s%s] %lld solves, %lld its (mean %.1f, max %lld)\n", prefix.c_str(), type.c_str(),
                (long long)stat_solves, (long long)stat_its, (double)stat_its / (double)stat_solves, (long long)stat_max);
}

void KSP::solve_gmres(const double *b, double *x, Ctx &c) {
    const int64_t mk = restart;
    const double haptol = 1e-30;
    std::vector<double> HH((mk + 1) * (mk + 1), 0.0), cc(mk + 1, 0.0), ss(mk + 1, 0.0), grs(mk + 2, 0.0),
        nrs(mk + 1, 0.0);
    auto H = [&](int64_t i, int64_t j) -> double & { return HH[(size_t)i * (mk + 1) + j]; };
    double *t1p = t1.p, *t2p = t2.p;
    launch_set(n, 0.0, x, c.st);
    its = 0;
    reason = 0;
    bool first = true;
    while (!reason) {
        double *v0 = V.p;
        if (first) {
            launch_copy(n, b, right ? v0 : t1p, c.st);
        } else {
            A->apply(x, t2p, c);
            launch_waxpby(n, 1.0, b, -1.0, t2p, right ? v0 : t1p, c.st);
        }
        if (!right) pc->apply(t1p, v0, c);
        double res = c.norm2(n, v0);
        history.push_back(res);
        if (monitor) { printf("  %3d KSP Residual norm %.12e\n", its, res); fflush(stdout); }
        if (res == 0.0) {
            reason = CONVERGED_ATOL;
            rnorm = 0.0;
            break;
        }
        launch_scale(n, 1.0 / res, v0, c.st);
        reason = converged(its, res);
        rnorm = res;
        std::fill(HH.begin(), HH.end(), 0.0);
        grs.assign(mk + 2, 0.0);
        grs[0] = res;
        int64_t loc_it = 0;
        while (!reason && loc_it < mk && its < maxit) {
            double *vk = V.p + loc_it * ldv;
            double *vn = V.p + (loc_it + 1) * ldv;
            if (right) {
                pc->apply(vk, t1p, c);
                A->apply(t1p, vn, c);
            } else {
                A->apply(vk, t1p, c);
                pc->apply(t1p, vn, c);
            }
            const int k = (int)(loc_it + 1);
            launch_mdot(n, k, nullptr, V.p, ldv, vn, c.partials(n, k), dh.p, c.st);
            c.comm->global_sum_dev(dh.p, k, c.st);
            launch_maxpy_norm(n, k, V.p, ldv, dh.p, -1.0, vn, c.partials(n, 1), dh.p + k, c.st);
            c.comm->global_sum_dev(dh.p + k, 1, c.st);
            double *hs = c.host_scalars(k + 1);
            HIPCHK(hipMemcpyAsync(hs, dh.p, sizeof(double) * (k + 1), hipMemcpyDeviceToHost, c.st));
            c.sync();
            for (int j = 0; j < k; ++j) H(j, loc_it) = hs[j];
            const double tt = std::sqrt(hs[k]);
            H(loc_it + 1, loc_it) = tt;
            double hapbnd = std::fabs(tt / grs[loc_it]);
            if (hapbnd > haptol) hapbnd = haptol;
            const bool hapend = tt < hapbnd;
            if (!hapend) launch_scale(n, 1.0 / tt, vn, c.st);
            // KSPGMRESUpdateHessenberg
            const int64_t it = loc_it;
            for (int64_t j = 0; j < it; ++j) {
                const double t0 = H(j, it);
                H(j, it) = cc[j] * t0 + ss[j] * H(j + 1, it);
                H(j + 1, it) = cc[j] * H(j + 1, it) - ss[j] * t0;
            }
            if (!hapend) {
                const double t0 = std::sqrt(H(it, it) * H(it, it) + H(it + 1, it) * H(it + 1, it));
                if (t0 == 0.0) {
                    reason = DIVERGED_NULL;
                    break;
                }
                cc[it] = H(it, it) / t0;
                ss[it] = H(it + 1, it) / t0;
                grs[it + 1] = -(ss[it] * grs[it]);
                grs[it] = cc[it] * grs[it];
                H(it, it) = cc[it] * H(it, it) + ss[it] * H(it + 1, it);
                res = std::fabs(grs[it + 1]);
            } else {
                res = 0.0;
            }
            loc_it++;
            its++;
            rnorm = res;
            history.push_back(res);
            if (monitor) { printf("  %3d KSP Residual norm %.12e\n", its, res); fflush(stdout); }
            reason = converged(its, res);
            if (hapend && !reason) {
                reason = DIVERGED_BREAKDOWN;
                break;
            }
        }
        // KSPGMRESBuildSoln
        const int64_t it = loc_it - 1;
        if (it >= 0) {
            if (H(it, it) == 0.0) {
                reason = DIVERGED_BREAKDOWN;
            } else {
                nrs[it] = grs[it] / H(it, it);
                for (int64_t k = it - 1; k >= 0; --k) {
                    double t0 = grs[k];
                    for (int64_t j = k + 1; j <= it; ++j) t0 = t0 - H(k, j) * nrs[j];
                    nrs[k] = t0 / H(k, k);
                }
                HIPCHK(hipMemcpyAsync(dh.p, nrs.data(), sizeof(double) * (it + 1), hipMemcpyHostToDevice, c.st));
                launch_lincomb(n, (int)(it + 1), V.p, ldv, dh.p, t2p, c.st);
                if (right) {
                    pc->apply(t2p, t1p, c);
                    launch_axpby(n, 1.0, t1p, 1.0, x, c.st);
                } else {
                    launch_axpby(n, 1.0, t2p, 1.0, x, c.st);
                }
                c.sync();  // nrs host buffer reuse
            }
        }
        if (its >= maxit) {
            if (!reason) reason = DIVERGED_ITS;
            break;
        }
        first = false;
    }
}

void KSP::solve_cg(const double *b, double *x, Ctx &c) {
    double *r = t1.p, *z = t2.p, *p = t3.p, *w = t4.p;
    launch_set(n, 0.0, x, c.st);
    launch_copy(n, b, r, c.st);
    double dp = 0.0;
    if (norm == "preconditioned") {
        pc->apply(r, z, c);
        dp = c.norm2(n, z);
    } else if (norm == "unpreconditioned") {
        dp = c.norm2(n, r);
    }
    history.push_back(dp);
    if (monitor) printf("  %3d KSP Residual norm %.12e\n", 0, dp);
    rnorm = dp;
    its = 0;
    reason = (norm != "none") ? converged(0, dp) : 0;
    if (reason) return;
    if (norm != "preconditioned") pc->apply(r, z, c);
    double beta = c.dot(n, z, r), betaold = 0.0, dpi = 0.0, dpiold = 0.0;
    int64_t i = 0;
    while (true) {
        its = (int)(i + 1);
        if (beta == 0.0) {
            reason = CONVERGED_ATOL;
            break;
        }
        // cg.c: (z, r) changing sign means an indefinite PC (e.g. ILU(0) of an
        // undrained solid block with negative pivots): stop with that reason
        // instead of iterating to max_it
        if (i > 0 && beta * betaold < 0.0) {
            reason = DIVERGED_INDEFINITE_PC;
            break;
        }
        if (i == 0) launch_copy(n, z, p, c.st);
        else launch_axpby(n, 1.0, z, beta / betaold, p, c.st);
        dpiold = dpi;
        A->apply(p, w, c);
        dpi = c.dot(n, p, w);
        betaold = beta;
        auto sgn = [](double v) { return (v > 0) - (v < 0); };
        if (dpi == 0.0 || (i > 0 && sgn(dpi) * sgn(dpiold) < 0)) {
            reason = DIVERGED_INDEFINITE_MAT;
            break;
        }
        const double a = beta / dpi;
        launch_axpby(n, a, p, 1.0, x, c.st);
        launch_axpby(n, -a, w, 1.0, r, c.st);
        if (norm == "preconditioned") {
            pc->apply(r, z, c);
            dp = c.norm2(n, z);
        } else if (norm == "unpreconditioned") {
            dp = c.norm2(n, r);
        } else {
            dp = 0.0;
        }
        rnorm = dp;
        history.push_back(dp);
        if (monitor) printf("  %3d KSP Residual norm %.12e\n", (int)(i + 1), dp);
        if (norm != "none") reason = converged((int)(i + 1), dp);
        if (reason) break;
        if (norm != "preconditioned") pc->apply(r, z, c);
        beta = c.dot(n, z, r);
        i++;
        if (i >= maxit) break;
    }
    if (i >= maxit && !reason) reason = DIVERGED_ITS;
}

// KSPSolve_CG with its scalar recurrences on the device (k_cg_state): the
// start (||r0||, the convergence test's reference, (z, r)) as in solve_cg,
// then iterations enqueued in batches -- 1 per read-back for the first 32,
// growing to 8 -- with one read-back of (done, its, reason) per batch instead
// of three scalar read-backs per iteration.  Iterations enqueued after the
// solve ended run their products and PC applies on frozen vectors (the vector
// updates and every state phase check the done flag): x, the iteration count,
// the reason and the history are those of solve_cg, bit for bit.
void KSP::solve_cg_dev(const double *b, double *x, Ctx &c) {
    double *r = t1.p, *z = t2.p, *p = t3.p, *w = t4.p;
    launch_set(n, 0.0, x, c.st);
    launch_copy(n, b, r, c.st);
    double dp = 0.0;
    if (norm == "preconditioned") {
        pc->apply(r, z, c);
        dp = c.norm2(n, z);
    } else if (norm == "unpreconditioned") {
        dp = c.norm2(n, r);
    }
    history.push_back(dp);
    if (monitor) printf("  %3d KSP Residual norm %.12e\n", 0, dp);
    rnorm = dp;
    its = 0;
    reason = (norm != "none") ? converged(0, dp) : 0;
    if (reason) return;
    if (norm != "preconditioned") pc->apply(r, z, c);
    const double beta0 = c.dot(n, z, r);
    if (cgS.n < (size_t)CG_NS) cgS.alloc(CG_NS);
    if (cgI.n < (size_t)CG_NI) cgI.alloc(CG_NI);
    if (cghist.n < (size_t)(maxit + 2)) cghist.alloc(maxit + 2);
    std::vector<double> hs(CG_NS, 0.0);
    hs[CG_BETA] = beta0;
    hs[CG_ONE] = 1.0;
    hs[CG_RNORM0] = rnorm0;
    hs[CG_TTOL] = ttol;
    std::vector<int64_t> hi(CG_NI, 0);
    HIPCHK(hipMemcpyAsync(cgS.p, hs.data(), sizeof(double) * CG_NS, hipMemcpyHostToDevice, c.st));
    HIPCHK(hipMemcpyAsync(cgI.p, hi.data(), sizeof(int64_t) * CG_NI, hipMemcpyHostToDevice, c.st));
    c.sync();  // (the host vectors above go out of scope only after the copies)
    const CgParams prm{rtol, atol, dtol, maxit, norm != "none" ? 1 : 0, CONVERGED_RTOL, CONVERGED_ATOL, DIVERGED_DTOL,
                       DIVERGED_NANORINF, DIVERGED_ITS, DIVERGED_INDEFINITE_PC, DIVERGED_INDEFINITE_MAT};
    double *S = cgS.p;
    int64_t *I = cgI.p;
    const int64_t *done = I + CG_DONE;
    auto sum_into = [&](const double *u, const double *v, double *slot) {
        launch_dot(n, u, v, c.partials(n, 1), slot, c.st);
        c.comm->global_sum_dev(slot, 1, c.st);
    };
    double *hb = c.host_scalars(CG_NI);
    int64_t i = 0;
    while (i < maxit) {
        // (at most 8 per batch: iterations enqueued past the end are wasted work --
        // batches of 32 cost more than the read-backs they saved, swelling N=80)
        const int64_t B = std::min<int64_t>(std::clamp<int64_t>(i / 16, 1, 8), maxit - i);
        for (int64_t k = 0; k < B; ++k, ++i) {
            launch_cg_state(CG_TOP, i, S, I, cghist.p, prm, c.st);
            if (i == 0) launch_copy(n, z, p, c.st);
            else launch_axpby_dev(n, S + CG_ONE, z, S + CG_BB, p, done, c.st);  // p = z + (beta / betaold) p
            A->apply(p, w, c);
            sum_into(p, w, S + CG_SLOT);
            launch_cg_state(CG_MID, i, S, I, cghist.p, prm, c.st);
            launch_axpby_dev(n, S + CG_A, p, S + CG_ONE, x, done, c.st);     // x += a p
            launch_axpby_dev(n, S + CG_NEGA, w, S + CG_ONE, r, done, c.st);  // r -= a w
            if (norm == "preconditioned") {
                pc->apply(r, z, c);
                sum_into(z, z, S + CG_SLOT);
            } else if (norm == "unpreconditioned") {
                sum_into(r, r, S + CG_SLOT);
            }
            launch_cg_state(CG_POST, i, S, I, cghist.p, prm, c.st);
            if (norm != "preconditioned") pc->apply(r, z, c);
            sum_into(z, r, S + CG_SLOT2);
            launch_cg_state(CG_END, i, S, I, cghist.p, prm, c.st);
        }
        HIPCHK(hipMemcpyAsync(hb, I, sizeof(int64_t) * CG_NI, hipMemcpyDeviceToHost, c.st));
        c.sync();
        int64_t d = 0;
        std::memcpy(&d, hb + CG_DONE, sizeof(d));
        if (d) break;
    }
    int64_t st[CG_NI];
    std::memcpy(st, hb, sizeof(st));
    its = (int)st[CG_ITS];
    reason = (int)st[CG_REASON];
    if (st[CG_HCOUNT] > 0) {
        std::vector<double> hh(st[CG_HCOUNT]);
        HIPCHK(hipMemcpyAsync(hh.data(), cghist.p, sizeof(double) * hh.size(), hipMemcpyDeviceToHost, c.st));
        c.sync();
        history.insert(history.end(), hh.begin(), hh.end());
        rnorm = hh.back();
    }
}

std::unique_ptr<KSP> make_ksp(const std::string &prefix, const Options &o, const DevCSR *Amat, const DevCSR *Pmat,
                              const std::string &default_ksp, const std::string &default_pc, Ctx &c, double rtol,
                              double atol, double dtol, int64_t maxit, int64_t restart, PC *external_pc) {
    auto k = std::make_unique<KSP>();
    k->prefix = prefix;
    k->type = o.str(prefix + "ksp_type", default_ksp);
    k->rtol = o.num(prefix + "ksp_rtol", rtol);
    k->atol = o.num(prefix + "ksp_atol", atol);
    k->dtol = o.num(prefix + "ksp_divtol", dtol);
    k->maxit = o.integer(prefix + "ksp_max_it", maxit);
    k->restart = o.integer(prefix + "ksp_gmres_restart", restart);
    k->monitor = o.has(prefix + "ksp_monitor");
    k->stats = o.flag("pls.ksp_stats", false);
    k->cg_device = o.flag("pls.cg_device", true);
    if (prefix == "global_") k->time_limit = o.num("pls.solver_time_limit", 0.0);
    if (o.has(prefix + "ksp_gmres_modifiedgramschmidt") && k->type == "gmres")
        throw Error(prefix + "ksp_gmres_modifiedgramschmidt: only classical Gram-Schmidt is implemented");
    k->resolve_side_norm(o.str(prefix + "ksp_pc_side", ""), o.str(prefix + "ksp_norm_type", ""));
    if (Amat) {
        k->owned_op = std::make_unique<MatOp>(Amat);
        k->A = k->owned_op.get();
        k->n = Amat->nrows;
    }
    if (external_pc) {
        k->pc = external_pc;
    } else {
        k->owned_pc = make_pc(o.str(prefix + "pc_type", default_pc), *Pmat, o, prefix, c);
        k->pc = k->owned_pc.get();
    }
    return k;
}

}  // namespace pls

namespace pls {

// =========================================================== fieldsplit ===
void upload(const HostCSR &H, DevCSR &M, Ctx &c) {
    upload_csr(M, H.nrows, H.ncols, H.rp.data(), H.ci.data(), H.v.data(), c);
}

// D2H of a matrix: the host arrays are allocated (zero-filled) on their own
// threads while the row pointers come over; big arrays then move through two
// pinned staging buffers, each chunk spread back by host threads (a pageable
// hipMemcpy of the N=59 s block's 5.1 GB ran at ~5 GB/s)
namespace {
// pinned staging buffers and their events, released on every path (a HIPCHK
// that throws mid-copy must not leak them: ADVICE r04)
struct Staging {
    void *buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    explicit Staging(size_t bytes) {
        for (int b = 0; b < 2; ++b) {
            HIPCHK(hipHostMalloc(&buf[b], bytes, hipHostMallocDefault));
            HIPCHK(hipEventCreateWithFlags(&ev[b], hipEventDisableTiming));
        }
    }
    ~Staging() {
        for (int b = 0; b < 2; ++b) {
            if (ev[b]) (void)hipEventDestroy(ev[b]);
            if (buf[b]) (void)hipHostFree(buf[b]);
        }
    }
    Staging(const Staging &) = delete;
    Staging &operator=(const Staging &) = delete;
};

void d2h_staged(void *dst, const void *src, size_t bytes, Ctx &c) {
    const size_t CH = (size_t)64 << 20;
    if (bytes < 2 * CH) {
        HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c.st));
        c.sync();
        return;
    }
    Staging S(CH);
    const size_t nch = (bytes + CH - 1) / CH;
    auto issue = [&](size_t k) {
        const size_t off = k * CH, len = std::min(CH, bytes - off);
        HIPCHK(hipMemcpyAsync(S.buf[k & 1], (const char *)src + off, len, hipMemcpyDeviceToHost, c.st));
        HIPCHK(hipEventRecord(S.ev[k & 1], c.st));
    };
    issue(0);
    const int T = 8;
    for (size_t k = 0; k < nch; ++k) {
        if (k + 1 < nch) issue(k + 1);  // (the other buffer: its copy-out finished below)
        HIPCHK(hipEventSynchronize(S.ev[k & 1]));
        const size_t off = k * CH, len = std::min(CH, bytes - off);
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                const size_t a = len * t / T, b = len * (t + 1) / T;
                std::memcpy((char *)dst + off + a, (const char *)S.buf[k & 1] + a, b - a);
            });
        for (auto &x : th) x.join();
    }
}
}  // namespace

HostCSR download(const DevCSR &M, Ctx &c) {
    HostCSR H;
    H.nrows = M.nrows;
    H.ncols = M.ncols;
    H.rp.resize(M.nrows + 1);
    {
        // (joined on every path: a HIPCHK that throws below must not destroy joinable threads)
        std::thread tci([&] { H.ci.resize(M.nnz); }), tv([&] { H.v.resize(M.nnz); });
        struct Join {
            std::thread &a, &b;
            ~Join() {
                if (a.joinable()) a.join();
                if (b.joinable()) b.join();
            }
        } join{tci, tv};
        HIPCHK(hipMemcpyAsync(H.rp.data(), M.rp.p, sizeof(int64_t) * (M.nrows + 1), hipMemcpyDeviceToHost, c.st));
        c.sync();
    }
    if (M.nnz) {
        d2h_staged(H.ci.data(), M.ci.p, sizeof(int32_t) * M.nnz, c);
        d2h_staged(H.v.data(), M.val.p, sizeof(double) * M.nnz, c);
    }
    return H;
}

namespace {
// rows `rows`, columns mapped by cmap (-1: dropped); cmap is monotone on the
// kept columns, so rows stay sorted (MatCreateSubMatrix with sorted ISs)
HostCSR submatrix(const HostCSR &M, const std::vector<int32_t> &rows, const std::vector<int32_t> &cmap,
                  int64_t ncols) {
    HostCSR S;
    S.nrows = (int64_t)rows.size();
    S.ncols = ncols;
    S.rp.assign(1, 0);
    for (int32_t r : rows) {
        for (int64_t k = M.rp[r]; k < M.rp[r + 1]; ++k) {
            const int32_t m = cmap[M.ci[k]];
            if (m >= 0) {
                S.ci.push_back(m);
                S.v.push_back(M.v[k]);
            }
        }
        S.rp.push_back((int64_t)S.ci.size());
    }
    return S;
}

// MatSchurComplementGetPmat, AINV_DIAG: D - C diag(A)^-1 B.  diag reciprocal
// keeps zeros (VecReciprocal); AinvB = row-scaled B; the product row i sums
// over k ascending (MatMatMult, sorted algorithm); then MatAYPX(S, -1, D).
HostCSR selfp(const HostCSR &A, const HostCSR &B, const HostCSR &C, const HostCSR &D) {
    std::vector<double> dinv(A.nrows, 0.0);
    for (int64_t i = 0; i < A.nrows; ++i)
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k)
            if (A.ci[k] == i) dinv[i] = A.v[k] != 0.0 ? 1.0 / A.v[k] : 0.0;
    std::vector<double> bs(B.v.size());
    for (int64_t i = 0; i < B.nrows; ++i)
        for (int64_t k = B.rp[i]; k < B.rp[i + 1]; ++k) bs[k] = dinv[i] * B.v[k];
    HostCSR S;
    S.nrows = D.nrows;
    S.ncols = D.ncols;
    std::vector<double> acc(D.ncols, 0.0);
    std::vector<char> mark(D.ncols, 0);
    std::vector<int32_t> cols;
    for (int64_t i = 0; i < C.nrows; ++i) {
        cols.clear();
        for (int64_t kk = C.rp[i]; kk < C.rp[i + 1]; ++kk) {
            const int32_t k = C.ci[kk];
            const double a = C.v[kk];
            for (int64_t jj = B.rp[k]; jj < B.rp[k + 1]; ++jj) {
                const int32_t j = B.ci[jj];
                if (!mark[j]) {
                    mark[j] = 1;
                    acc[j] = 0.0;
                    cols.push_back(j);
                }
                acc[j] += a * bs[jj];
            }
        }
        for (int64_t kk = D.rp[i]; kk < D.rp[i + 1]; ++kk)
            if (!mark[D.ci[kk]]) {
                mark[D.ci[kk]] = 2;  // D only
                cols.push_back(D.ci[kk]);
            }
        std::sort(cols.begin(), cols.end());
        int64_t dk = D.rp[i];
        for (int32_t j : cols) {
            double dv = 0.0;
            bool hasd = false;
            while (dk < D.rp[i + 1] && D.ci[dk] < j) ++dk;
            if (dk < D.rp[i + 1] && D.ci[dk] == j) {
                dv = D.v[dk];
                hasd = true;
            }
            double out;
            if (mark[j] == 2) out = dv;
            else out = hasd ? dv - acc[j] : -acc[j];
            S.ci.push_back(j);
            S.v.push_back(out);
            mark[j] = 0;
        }
        S.rp.push_back((int64_t)S.ci.size());
    }
    return S;
}


// S x = A11 x - A10 A00^-1 A01 x (MatMult_SchurComplement; inner solve = the split-0 KSP)
struct SchurOp : Op {
    const DevCSR *A01, *A10, *A11;
    KSP *k0;
    DBuf<double> w1, w2, w3;
    SchurOp(const DevCSR *a01, const DevCSR *a10, const DevCSR *a11, KSP *k) : A01(a01), A10(a10), A11(a11), k0(k) {
        n = a11->nrows;
        w1.alloc(std::max<int64_t>(a01->nrows, 1));
        w2.alloc(std::max<int64_t>(a01->nrows, 1));
        w3.alloc(std::max<int64_t>(n, 1));
    }
    void apply(const double *x, double *y, Ctx &c) override {
        spmv(*A01, x, w1.p, c);
        k0->solve(w1.p, w2.p, c);
        spmv(*A10, w2.p, w3.p, c);
        spmv(*A11, x, y, c, 1.0, -1.0, w3.p);
    }
};
}  // namespace

PCFieldSplit::PCFieldSplit(const DevCSR &M, const std::vector<int32_t> &s0, const std::vector<int32_t> &s1,
                           const Options &o, const std::string &prefix, Ctx &c) {
    type = "fieldsplit";
    n = M.nrows;
    if (M.halo) throw Error(prefix + "pc_type fieldsplit: not available with several ranks");
    n0 = (int64_t)s0.size();
    n1 = (int64_t)s1.size();
    if (n0 == 0 || n1 == 0 || n0 + n1 != n)
        throw Error(prefix + "pc_type fieldsplit: the two splits must be non-empty and cover the block (" +
                    std::to_string(n0) + " + " + std::to_string(n1) + " of " + std::to_string(n) + " rows)");
    ftype = o.str(prefix + "pc_fieldsplit_type", "multiplicative");
    if (ftype != "additive" && ftype != "multiplicative" && ftype != "schur")
        throw Error(prefix + "pc_fieldsplit_type " + ftype + " is not available (additive, multiplicative, schur)");
    const HostCSR Mh = download(M, c);
    std::vector<int32_t> m0(n, -1), m1(n, -1);
    for (int64_t i = 0; i < n0; ++i) m0[s0[i]] = (int32_t)i;
    for (int64_t i = 0; i < n1; ++i) m1[s1[i]] = (int32_t)i;
    const HostCSR h00 = submatrix(Mh, s0, m0, n0), h01 = submatrix(Mh, s0, m1, n1);
    const HostCSR h10 = submatrix(Mh, s1, m0, n0), h11 = submatrix(Mh, s1, m1, n1);
    upload(h00, A00, c);
    upload(h01, A01, c);
    upload(h10, A10, c);
    upload(h11, A11, c);
    for (DevCSR *B : {&A01, &A10, &A11}) build_sell(*B, c);
    const std::string p0 = prefix + "fieldsplit_0_", p1 = prefix + "fieldsplit_1_";
    k0 = make_ksp(p0, o, &A00, &A00, "preonly", "ilu", c);
    if (ftype == "schur") {
        fact = o.str(prefix + "pc_fieldsplit_schur_fact_type", "full");
        if (fact != "diag" && fact != "lower" && fact != "upper" && fact != "full")
            throw Error(prefix + "pc_fieldsplit_schur_fact_type " + fact + " is not available");
        scale = o.num(prefix + "pc_fieldsplit_schur_scale", -1.0);
        const std::string pre = o.str(prefix + "pc_fieldsplit_schur_precondition", "a11");
        const DevCSR *pmat = &A11;
        if (pre == "selfp") {
            upload(selfp(h00, h01, h10, h11), Sp, c);
            pmat = &Sp;
        } else if (pre != "a11") {
            throw Error(prefix + "pc_fieldsplit_schur_precondition " + pre + " is not available (selfp, a11)");
        }
        k1 = make_ksp(p1, o, nullptr, pmat, "gmres", "ilu", c);
        k1->owned_op = std::make_unique<SchurOp>(&A01, &A10, &A11, k0.get());
        k1->A = k1->owned_op.get();
        k1->n = n1;
    } else {
        k1 = make_ksp(p1, o, &A11, &A11, "preonly", "ilu", c);
    }
    for (auto *b : {&x0, &y0, &t0}) b->alloc(std::max<int64_t>(n0, 1));
    for (auto *b : {&x1, &y1, &t1}) b->alloc(std::max<int64_t>(n1, 1));
    is0.alloc(std::max<int64_t>(n0, 1));
    is1.alloc(std::max<int64_t>(n1, 1));
    if (n0) HIPCHK(hipMemcpyAsync(is0.p, s0.data(), sizeof(int32_t) * n0, hipMemcpyHostToDevice, c.st));
    if (n1) HIPCHK(hipMemcpyAsync(is1.p, s1.data(), sizeof(int32_t) * n1, hipMemcpyHostToDevice, c.st));
    c.sync();
}

// PCApply_FieldSplit / PCApply_FieldSplit_Schur
void PCFieldSplit::apply(const double *x, double *y, Ctx &c) {
    launch_pack(n0, is0.p, x, x0.p, c.st);
    launch_pack(n1, is1.p, x, x1.p, c.st);
    auto x1_minus_A10 = [&](const double *v) { spmv(A10, v, t1.p, c, -1.0, 1.0, x1.p); };   // t1 = x1 - A10 v
    auto x0_minus_A01 = [&](const double *v) { spmv(A01, v, t0.p, c, -1.0, 1.0, x0.p); };   // t0 = x0 - A01 v
    if (ftype == "additive") {
        k0->solve(x0.p, y0.p, c);
        k1->solve(x1.p, y1.p, c);
    } else if (ftype == "multiplicative" || fact == "lower") {
        k0->solve(x0.p, y0.p, c);
        x1_minus_A10(y0.p);
        k1->solve(t1.p, y1.p, c);
    } else if (fact == "diag") {
        k0->solve(x0.p, y0.p, c);
        k1->solve(x1.p, y1.p, c);
        launch_scale(n1, scale, y1.p, c.st);
    } else if (fact == "upper") {
        k1->solve(x1.p, y1.p, c);
        x0_minus_A01(y1.p);
        k0->solve(t0.p, y0.p, c);
    } else {  // full
        k0->solve(x0.p, y0.p, c);
        x1_minus_A10(y0.p);
        k1->solve(t1.p, y1.p, c);
        x0_minus_A01(y1.p);
        k0->solve(t0.p, y0.p, c);
    }
    launch_unpack(n0, is0.p, y0.p, y, c.st);
    launch_unpack(n1, is1.p, y1.p, y, c.st);
}

}  // namespace pls
