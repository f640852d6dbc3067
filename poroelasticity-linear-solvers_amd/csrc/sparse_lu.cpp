// sparse_lu.cpp -- exact sparse LU (PCLU) of large blocks: nested dissection +
// a multifrontal factorization on the device.  The MUMPS stand-in for blocks
// too large for the dense inverse (dense.hip): the reference factors every
// block with MUMPS in petsc-options-exact:11-35 and the Schur split of the fp
// fieldsplit in petsc-options-inexact:98-106.
//
// Ordering.  Nested dissection of the symmetrized graph (George's automatic
// nested dissection): a breadth-first level structure from a pseudo-peripheral
// vertex; the separator is the smallest level set whose two sides each hold
// 30-70 % of the vertices; recursion on both sides down to `leaf` vertices; a
// set the search does not connect splits into its components (empty separator).
// The dissection tree is the assembly tree: a node's pivots are its separator
// (or leaf) vertices, numbered in postorder, so every subtree is contiguous and
// a node's update rows (its "structure") are vertices of its ancestors.
//
// Factorization.  Level by level from the deepest: every front of a level is a
// dense (p + q)^2 block (padded to 64) assembled from the original entries
// whose earlier-eliminated index is one of its pivots and the extend-add of its
// children's update blocks; a partial Gauss-Jordan elimination of the p pivot
// columns (64 x 64 tiles, no pivoting, like the dense and band LU) leaves
//     [ F11^-1       F11^-1 F12           ]
//     [ -F21 F11^-1  F22 - F21 F11^-1 F12 ]
// whose last block is the update passed to the parent.  The first two blocks
// are kept (the "U part", p x (p + q)) and the bottom-left one (the "X part").
// The LU is exact up to rounding (ordering-invariant in exact arithmetic, as
// MUMPS reorders too).
//
// Solve.  Forward, deepest level first: z_p = b_p + the children's
// contributions at the front's rows, the front's contribution to its update
// rows cu = (children's) + X z_p; backward, root first: x_p = F11^-1 z_p -
// (F11^-1 F12) x_q.  Every level is three batched launches (a gather and two
// wave-per-row GEMVs over the stored factors), so one apply reads the factors
// once at HBM rate with ~3 launches per tree level.  All sums run in a fixed
// order (children in tree order): the result does not depend on timing.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <numeric>

#include "nd_order.hpp"
#include "runtime.hpp"

namespace pls {

// Ordering + symbolic analysis (host): the dissection tree, pivots numbered in
// postorder, every front's update rows (ND positions, ascending).
struct LUSymbolic {
    NDTree T;
    std::vector<int32_t> post, pos, permh, front_of;
    std::vector<int64_t> pstart;
    std::vector<std::vector<int32_t>> st;
    std::vector<int64_t> gp;
    std::vector<int32_t> gi;
    int64_t nfront = 0, nlevels = 0;
    double t_order = 0, t_symbolic = 0;
};

NDOptions lu_nd_options(const Options &o) {
    NDOptions nd;
    nd.leaf = std::max<int64_t>(1, o.integer("pls.lu_nd_leaf", 64));
    nd.method = (int)o.integer("pls.lu_nd", 1);
    nd.imbalance = o.num("pls.lu_nd_imbalance", 1.10);
    nd.seeds = (int)o.integer("pls.lu_nd_seeds", 6);
    nd.compress = o.flag("pls.lu_nd_compress", true);
    nd.node_passes = (int)o.integer("pls.lu_nd_node_passes", 4);
    nd.threads = (int)o.integer("pls.lu_nd_threads", 0);
    return nd;
}

namespace {

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// ND positions, pivot ranges and update rows of every front from the tree's
// pivot sets (Y.T.piv) in postorder; re-run after delayed pivots moved
// variables to their parents' fronts
void lu_structure(LUSymbolic &Y) {
    const NDTree &T = Y.T;
    const int64_t n = (int64_t)Y.pos.size();
    const double t1 = now_s();
    Y.pstart.assign(Y.nfront, 0);
    {
        int64_t k = 0;
        for (int32_t f : Y.post) {
            Y.pstart[f] = k;
            for (int32_t v : T.piv[f]) {
                Y.pos[v] = (int32_t)k;
                Y.permh[k] = v;
                Y.front_of[k] = f;
                ++k;
            }
        }
        if (k != n) throw Error("lu: the dissection does not cover every row");
    }
    // update rows (ND positions, ascending) of every front
    Y.st.assign(Y.nfront, {});
    {
        std::vector<int32_t> mark(n, -1);
        for (int32_t f : Y.post) {
            const int64_t pend = Y.pstart[f] + (int64_t)T.piv[f].size();
            std::vector<int32_t> &s = Y.st[f];
            auto add = [&](int32_t p) {
                if (p >= pend && mark[p] != f) {
                    mark[p] = f;
                    s.push_back(p);
                }
            };
            for (int32_t cch : T.ch[f])
                for (int32_t p : Y.st[cch]) add(p);
            for (int32_t v : T.piv[f])
                for (int64_t k = Y.gp[v]; k < Y.gp[v + 1]; ++k) add(Y.pos[Y.gi[k]]);
            std::sort(s.begin(), s.end());
        }
    }
    Y.t_symbolic += now_s() - t1;
}

LUSymbolic lu_symbolic(const HostCSR &A, const Options &o) {
    LUSymbolic Y;
    const int64_t n = A.nrows;
    const double t0 = now_s();
    sym_graph(A, Y.gp, Y.gi, true);  // stored zeros are not structure: they add no fill
    Y.T = nested_dissection(Y.gp, Y.gi, n, lu_nd_options(o));
    const NDTree &T = Y.T;
    Y.nfront = (int64_t)T.piv.size();
    // postorder: children before parents, subtrees contiguous
    Y.post.reserve(Y.nfront);
    {
        std::vector<std::pair<int32_t, int32_t>> stk{{0, 0}};
        while (!stk.empty()) {
            auto &[v, k] = stk.back();
            if (k < (int32_t)T.ch[v].size()) {
                const int32_t cch = T.ch[v][k++];
                stk.push_back({cch, 0});
            } else {
                Y.post.push_back(v);
                stk.pop_back();
            }
        }
    }
    Y.pos.assign(n, 0);
    Y.permh.assign(n, 0);
    Y.front_of.assign(n, 0);
    Y.t_order = now_s() - t0;
    Y.t_symbolic = 0;
    lu_structure(Y);
    int32_t maxd = 0;
    for (int32_t d : T.depth) maxd = std::max(maxd, d);
    Y.nlevels = maxd + 1;
    return Y;
}

// Host-only analysis (pls_sparse_lu_analyze): sizes of the factorization the
// options would build.  stats: n, fronts, levels, largest front (p + q),
// factor doubles read per solve sum p (p + 2 q), doubles stored (padded layout),
// factorization flops, ordering s, symbolic s, largest separator p
void sparse_lu_analyze(const HostCSR &A, const Options &o, double *stats, int64_t nstats, int32_t *perm,
                       int32_t *front_of, int32_t *parent) {
    const LUSymbolic Y = lu_symbolic(A, o);
    std::vector<int32_t> pnum(Y.nfront);  // postorder number of every front
    for (size_t k = 0; k < Y.post.size(); ++k) pnum[Y.post[k]] = (int32_t)k;
    for (int64_t k = 0; k < A.nrows; ++k) {
        if (perm) perm[k] = Y.permh[k];
        if (front_of) front_of[k] = pnum[Y.front_of[k]];
    }
    if (parent)
        for (int32_t f = 0; f < (int32_t)Y.nfront; ++f)
            parent[pnum[f]] = Y.T.parent[f] < 0 ? -1 : pnum[Y.T.parent[f]];
    double v[10] = {(double)A.nrows, (double)Y.nfront, (double)Y.nlevels, 0, 0, 0, 0, Y.t_order, Y.t_symbolic, 0};
    for (int32_t f = 0; f < (int32_t)Y.nfront; ++f) {
        const double p = (double)Y.T.piv[f].size(), q = (double)Y.st[f].size();
        const double pp = std::ceil(p / 64) * 64, ld = pp + std::ceil(q / 64) * 64;
        v[3] = std::max(v[3], p + q);
        v[4] += p * (p + 2 * q);  // compact U (p x (p + q)) and X (q x p) parts: stored and read once per solve
        v[5] += ld * ld;          // the front's dense workspace during the factorization (tiles padded)
        (void)pp;
        v[6] += 2.0 / 3.0 * p * p * p + 2.0 * p * p * q + 2.0 * p * q * q;
        v[9] = std::max(v[9], p);
    }
    for (int64_t k = 0; k < std::min<int64_t>(nstats, 10); ++k) stats[k] = v[k];
}

struct PCSparseLU : PC {
    int64_t nfront = 0, nlevels = 0;
    DBuf<int32_t> perm;   // ND position -> unknown (column) of M: the solution's scatter
    DBuf<int32_t> rperm;  // ND position -> equation (row) of M after threshold pivoting: the right-hand side's gather
    int32_t piv_stats[3] = {0, 0, 0};  // rows exchanged, pivots below u x column max, zero columns
    double piv_u = 0.0;
    DBuf<double> U, X;   // factors (per front: U part pp x ld, X part q x pp)
    DBuf<MSolve> S;
    DBuf<int32_t> slist;
    // per level: fronts' rows for the solve kernels (level offsets on the host)
    DBuf<int32_t> rf, rl, qf, ql, pf, pl;
    DBuf<int64_t> cptr, cidx;
    std::vector<int64_t> lr_off, lq_off, lp_off;  // nlevels + 1
    std::map<hipStream_t, std::unique_ptr<DBuf<double>>> work;  // per stream: bp, z, x, cu, acc
    int64_t nq = 0;
    double setup_s[4] = {0, 0, 0, 0};  // ordering, symbolic, factorization, total
    double factor_gb = 0;
    int static_pivots = 0;
    double tau_used = 0.0;  // the static pivoting threshold applied

    int delayed = 0, delay_rounds = 0;  // variables moved to their parents' fronts, re-analyses
    int64_t maxf = 0;                   // largest front (p + q)

    PCSparseLU(const DevCSR &M, const Options &o, Ctx &c) {
        type = "lu";
        n = M.nrows;
        if (M.ncols != n) throw Error("lu: block is not square");
        const double t0 = now_s();
        const HostCSR A = download(M, c);
        LUSymbolic Y = lu_symbolic(A, o);
        // Delayed pivots (MUMPS): a column whose best fully-summed candidate is below
        // u x its largest entry over the front (update rows included) is not
        // eliminated in this front but in its parent's, where the rows that made it
        // small are fully summed too.  Here that is a re-analysis: the flagged
        // variables move to their parents' pivot sets, the structure is recomputed
        // and the factorization re-run (pls.lu_delay_rounds times at most; 0: off,
        // the best candidate is used as it is).  The root's columns cannot move.
        const int64_t rounds = o.integer("pls.lu_delay_rounds", 8);
        for (int round = 0;; ++round) {
            std::vector<int32_t> dfl;
            factor(M, A, Y, o, c, t0, round < rounds ? &dfl : nullptr);
            int moved = 0;
            for (int64_t i = 0; i < (int64_t)dfl.size(); ++i) {
                if (!dfl[i]) continue;
                const int32_t f = Y.front_of[i], g = Y.T.parent[f], v = Y.permh[i];
                if (g < 0) continue;
                auto &pf = Y.T.piv[f];
                pf.erase(std::find(pf.begin(), pf.end(), v));
                Y.T.piv[g].push_back(v);
                ++moved;
            }
            if (!moved) break;
            delayed += moved;
            ++delay_rounds;
            lu_structure(Y);
        }
        setup_s[3] = now_s() - t0;
        if (o.flag("pls.lu_view", false))
            fprintf(stderr,
                    "[sparse lu] n %lld: %lld fronts, %lld levels, largest front %lld, factors %.2f GB, %d static "
                    "pivots, refinement steps %d; threshold pivoting u = %g: %d rows exchanged, %d pivots below u x "
                    "column max, %d zero columns; %d delayed pivots (%d re-analyses); setup: ordering %.2f s, "
                    "symbolic %.2f s, factorization %.2f s, total %.2f s\n",
                    (long long)n, (long long)nfront, (long long)nlevels, (long long)maxf, factor_gb, static_pivots,
                    refine, piv_u, piv_stats[0], piv_stats[1], piv_stats[2], delayed, delay_rounds, setup_s[0],
                    setup_s[1], setup_s[2], setup_s[3]);
    }

    // numeric factorization and solve tables for the structure Y; dfl (if given):
    // per ND position 1 where the column's pivot fell below the threshold
    void factor(const DevCSR &M, const HostCSR &A, LUSymbolic &Y, const Options &o, Ctx &c, double t0,
                std::vector<int32_t> *dfl) {
        const NDTree &T = Y.T;
        nfront = Y.nfront;
        const std::vector<int32_t> &post = Y.post, &pos = Y.pos, &permh = Y.permh, &front_of = Y.front_of;
        const std::vector<int64_t> &pstart = Y.pstart;
        const std::vector<std::vector<int32_t>> &st = Y.st;
        const double t1 = t0 + Y.t_order;
        // ---- sizes, levels
        int32_t maxd = 0;
        for (int32_t d : T.depth) maxd = std::max(maxd, d);
        nlevels = maxd + 1;
        std::vector<std::vector<int32_t>> bylev(nlevels);
        for (int32_t f : post) bylev[T.depth[f]].push_back(f);
        std::vector<int64_t> p(nfront), q(nfront), pp(nfront), ld(nfront), uoff(nfront), xoff(nfront), soff(nfront),
            qoff(nfront);
        int64_t usz = 0, xsz = 0, ssz = 0;
        for (int32_t f : post) {
            p[f] = (int64_t)T.piv[f].size();
            q[f] = (int64_t)st[f].size();
            pp[f] = (p[f] + 63) / 64 * 64;
            ld[f] = pp[f] + (q[f] + 63) / 64 * 64;
            uoff[f] = usz;  // compact: U part p x (p + q), X part q x p (no tile padding)
            usz += p[f] * (p[f] + q[f]);
            xoff[f] = xsz;
            xsz += q[f] * p[f];
            soff[f] = qoff[f] = ssz;
            ssz += q[f];
        }
        nq = ssz;
        factor_gb = (double)(usz + xsz) * 8e-9;
        const double cap = o.num("pls.lu_sparse_max_gb", 1e9);
        if (factor_gb > cap)
            throw Error("lu: sparse factors need " + std::to_string(factor_gb) + " GB (pls.lu_sparse_max_gb)");
        U.alloc(std::max<int64_t>(usz, 1));
        X.alloc(std::max<int64_t>(xsz, 1));
        // row of an ND position inside front f's dense block: pivots [0, p), update
        // rows from pp on (the pivot block is padded to whole tiles)
        auto local = [&](int32_t f, int32_t ppos) -> int64_t {
            if (ppos >= pstart[f] && ppos < pstart[f] + p[f]) return ppos - pstart[f];
            const auto &s = st[f];
            const auto it = std::lower_bound(s.begin(), s.end(), ppos);
            if (it == s.end() || *it != ppos) throw Error("lu: sparse symbolic structure is inconsistent");
            return pp[f] + (it - s.begin());
        };
        // extend-add maps: child's update rows -> parent's local rows
        std::vector<int32_t> maps(std::max<int64_t>(ssz, 1));
        for (int32_t f : post)
            if (T.parent[f] >= 0)
                for (int64_t k = 0; k < q[f]; ++k) maps[soff[f] + k] = (int32_t)local(T.parent[f], st[f][k]);
        // original entries: owner = the front of the earlier-eliminated index
        std::vector<std::vector<int64_t>> sc_dst(nlevels), sc_src(nlevels);
        std::vector<int64_t> wsoff(nfront), lev_ws(nlevels, 0);
        for (int64_t d = 0; d < nlevels; ++d)
            for (int32_t f : bylev[d]) {
                wsoff[f] = lev_ws[d];
                lev_ws[d] += ld[f] * ld[f];
            }
        for (int64_t i = 0; i < n; ++i)
            for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                if (A.v[k] == 0.0 && A.ci[k] != i) continue;  // stored zero: outside the (value) structure
                const int32_t pi = pos[i], pj = pos[A.ci[k]];
                const int32_t f = front_of[std::min(pi, pj)];
                const int64_t r = local(f, pi), cc = local(f, pj);
                sc_dst[T.depth[f]].push_back(wsoff[f] + r * ld[f] + cc);
                sc_src[T.depth[f]].push_back(k);
            }
        const double t2 = now_s();
        // ---- numeric factorization, deepest level first
        int64_t wsmax = 1;
        for (int64_t d = 0; d < nlevels; ++d) wsmax = std::max(wsmax, lev_ws[d]);
        DBuf<double> Wa(wsmax), Wb(wsmax), val(std::max<int64_t>(M.nnz, 1));
        HIPCHK(hipMemcpyAsync(val.p, A.v.data(), sizeof(double) * A.v.size(), hipMemcpyHostToDevice, c.st));
        DBuf<int32_t> dmaps(maps.size()), fail(2);
        HIPCHK(hipMemcpyAsync(dmaps.p, maps.data(), sizeof(int32_t) * maps.size(), hipMemcpyHostToDevice, c.st));
        HIPCHK(hipMemsetAsync(fail.p, 0, sizeof(int32_t) * 2, c.st));
        // static pivoting threshold: pls.lu_static_pivot x max |a_ij|; 0 (default, MUMPS's
        // CNTL(4) <= 0): off, an exactly zero pivot is an error
        double amax = 0.0;
        for (double v : A.v) amax = std::max(amax, std::fabs(v));
        const double tau = o.num("pls.lu_static_pivot", 0.0) * amax;
        tau_used = tau;
        // threshold partial pivoting over each front's fully-summed rows (MUMPS CNTL(1) = u,
        // pls.lu_pivot_threshold, default 0.01; 0: pivots only inside each 64 x 64 tile)
        const double u = o.num("pls.lu_pivot_threshold", 0.01);
        piv_u = u;
        DBuf<int32_t> drowp(std::max<int64_t>(n, 1)), pstats(3), dflag(dfl ? std::max<int64_t>(n, 1) : 0);
        if (dfl) HIPCHK(hipMemsetAsync(dflag.p, 0, sizeof(int32_t) * std::max<int64_t>(n, 1), c.st));
        {
            std::vector<int32_t> lid(std::max<int64_t>(n, 1), 0);
            for (int32_t f : post)
                for (int64_t r = 0; r < p[f]; ++r) lid[pstart[f] + r] = (int32_t)r;
            HIPCHK(hipMemcpyAsync(drowp.p, lid.data(), sizeof(int32_t) * lid.size(), hipMemcpyHostToDevice, c.st));
            HIPCHK(hipMemsetAsync(pstats.p, 0, sizeof(int32_t) * 3, c.st));
            c.sync();
        }
        double *Wcur = Wa.p, *Wprev = Wb.p;
        std::vector<int64_t> prev_ws;  // workspace offsets of the previous (deeper) level's fronts
        constexpr int CH = 32768;      // fronts per batched launch (grid z / y limit)
        for (int64_t d = nlevels - 1; d >= 0; --d) {
            const auto &fl = bylev[d];
            HIPCHK(hipMemsetAsync(Wcur, 0, sizeof(double) * lev_ws[d], c.st));
            for (size_t c0 = 0; c0 < fl.size(); c0 += CH) {
                const size_t c1 = std::min(fl.size(), c0 + CH);
                std::vector<MFront> hf;
                std::vector<MStore> hs;
                int max_pad = 0, max_ldt = 0, max_rows = 0, max_pt = 0;
                for (size_t t = c0; t < c1; ++t) {
                    const int32_t f = fl[t];
                    hf.push_back({wsoff[f], (int32_t)(ld[f] / 64), (int32_t)(pp[f] / 64), (int32_t)p[f], (int32_t)q[f]});
                    hs.push_back({uoff[f], xoff[f]});
                    max_pad = std::max(max_pad, (int)(pp[f] - p[f]));
                    max_ldt = std::max(max_ldt, (int)(ld[f] / 64));
                    max_pt = std::max(max_pt, (int)(pp[f] / 64));
                    max_rows = std::max(max_rows, (int)(pp[f] + q[f]));
                }
                DBuf<MFront> dF(hf.size());
                DBuf<MStore> dS(hs.size());
                DBuf<double> Dt(hf.size() * 4096);
                HIPCHK(hipMemcpyAsync(dF.p, hf.data(), sizeof(MFront) * hf.size(), hipMemcpyHostToDevice, c.st));
                HIPCHK(hipMemcpyAsync(dS.p, hs.data(), sizeof(MStore) * hs.size(), hipMemcpyHostToDevice, c.st));
                // threshold pivoting: per front its pivot rows' offset in rowperm and a (p + q) x 64 panel scratch
                std::vector<int64_t> hpst, hsoff;
                int64_t pscr = 0;
                for (size_t t = c0; t < c1; ++t) {
                    const int32_t f = fl[t];
                    hpst.push_back(pstart[f]);
                    hsoff.push_back(pscr);
                    pscr += (p[f] > 1 || (p[f] == 1 && q[f] > 0) ? p[f] + q[f] : 0) * 64;
                }
                DBuf<int64_t> dpst(hpst.size()), dsoff(hsoff.size());
                int64_t max_pq = 0;
                for (size_t t = c0; t < c1; ++t) max_pq = std::max<int64_t>(max_pq, p[fl[t]] + q[fl[t]]);
                // (then the panels' fast-path scratch, one per front)
                DBuf<double> Pscr(u > 0.0 ? pscr + (int64_t)(c1 - c0) * panel_fast_doubles() : 1);
                HIPCHK(hipMemcpyAsync(dpst.p, hpst.data(), sizeof(int64_t) * hpst.size(), hipMemcpyHostToDevice, c.st));
                HIPCHK(hipMemcpyAsync(dsoff.p, hsoff.data(), sizeof(int64_t) * hsoff.size(), hipMemcpyHostToDevice,
                                      c.st));
                launch_mf_pad((int)hf.size(), dF.p, max_pad, Wcur, c.st);
                if (c0 == 0) {  // the level's original entries (all of its fronts)
                    DBuf<int64_t> dd(std::max<size_t>(sc_dst[d].size(), 1)), ds(std::max<size_t>(sc_src[d].size(), 1));
                    HIPCHK(hipMemcpyAsync(dd.p, sc_dst[d].data(), sizeof(int64_t) * sc_dst[d].size(), hipMemcpyHostToDevice,
                                          c.st));
                    HIPCHK(hipMemcpyAsync(ds.p, sc_src[d].data(), sizeof(int64_t) * sc_src[d].size(), hipMemcpyHostToDevice,
                                          c.st));
                    launch_mf_scatter((int64_t)sc_dst[d].size(), dd.p, ds.p, val.p, Wcur, c.st);
                    c.sync();  // dd / ds are freed below
                    // extend-add, one child rank per launch (children of a parent never race)
                    size_t maxch = 0;
                    for (int32_t f : fl) maxch = std::max(maxch, T.ch[f].size());
                    for (size_t r = 0; r < maxch; ++r) {
                        std::vector<MChild> hc;
                        int max_q = 0;
                        for (int32_t f : fl)
                            if (r < T.ch[f].size()) {
                                const int32_t cf = T.ch[f][r];
                                if (q[cf] == 0) continue;
                                hc.push_back({prev_ws[cf], wsoff[f], soff[cf], (int32_t)ld[cf], (int32_t)pp[cf],
                                              (int32_t)ld[f], (int32_t)q[cf]});
                                max_q = std::max(max_q, (int)q[cf]);
                            }
                        for (size_t h0 = 0; h0 < hc.size(); h0 += CH) {
                            const size_t h1 = std::min(hc.size(), h0 + CH);
                            DBuf<MChild> dC(h1 - h0);
                            HIPCHK(hipMemcpyAsync(dC.p, hc.data() + h0, sizeof(MChild) * (h1 - h0), hipMemcpyHostToDevice,
                                                  c.st));
                            launch_mf_extend((int)(h1 - h0), dC.p, max_q, dmaps.p, Wprev, Wcur, c.st);
                            c.sync();
                        }
                    }
                }
                for (int k = 0; k < max_pt; ++k) {
                    launch_mf_panel_pivot((int)hf.size(), dF.p, dpst.p, dsoff.p, k, Wcur, Pscr.p, drowp.p, pstats.p, u,
                                          c.st, dflag.p, u > 0.0 ? Pscr.p + pscr : nullptr, max_pq);
                    launch_mf_gj_step((int)hf.size(), dF.p, max_ldt, k, Wcur, Dt.p, fail.p, tau, c.st);
                }
                launch_mf_store((int)hf.size(), dF.p, dS.p, max_rows, Wcur, U.p, X.p, c.st);
                HIPCHK(hipGetLastError());
                c.sync();
            }
            prev_ws.assign(nfront, 0);
            for (int32_t f : fl) prev_ws[f] = wsoff[f];
            std::swap(Wcur, Wprev);
        }
        int32_t hfail[2] = {0, 0};
        HIPCHK(hipMemcpyAsync(hfail, fail.p, sizeof(int32_t) * 2, hipMemcpyDeviceToHost, c.st));
        std::vector<int32_t> rowp(std::max<int64_t>(n, 1));
        HIPCHK(hipMemcpyAsync(rowp.data(), drowp.p, sizeof(int32_t) * rowp.size(), hipMemcpyDeviceToHost, c.st));
        HIPCHK(hipMemcpyAsync(piv_stats, pstats.p, sizeof(int32_t) * 3, hipMemcpyDeviceToHost, c.st));
        if (dfl) {
            dfl->assign(std::max<int64_t>(n, 1), 0);
            HIPCHK(hipMemcpyAsync(dfl->data(), dflag.p, sizeof(int32_t) * dfl->size(), hipMemcpyDeviceToHost, c.st));
        }
        c.sync();
        if (dfl) {  // delays pending: this factorization is replaced; a zero pivot here is not final
            bool any = false;
            for (int64_t i = 0; i < n && !any; ++i) any = (*dfl)[i] && T.parent[Y.front_of[i]] >= 0;
            if (any) return;
        }
        if (hfail[0]) throw Error("LU: zero pivot (PETSc: MAT_FACTOR_NUMERIC_ZEROPIVOT)");
        // the equations' order after the exchanges: ND position -> row of M
        std::vector<int32_t> rpermh(std::max<int64_t>(n, 1));
        for (int64_t i = 0; i < n; ++i) rpermh[i] = permh[pstart[front_of[i]] + rowp[i]];
        static_pivots = hfail[1];
        const double t3 = now_s();
        // ---- solve tables
        std::vector<MSolve> hS(nfront);
        std::vector<int32_t> hsl(std::max<int64_t>(ssz, 1));
        for (int32_t f : post) {
            // compact factors: X rows are p long, U rows p + q (the kernels' "pp" / "ld")
            hS[f] = {pstart[f], qoff[f], uoff[f], xoff[f], soff[f], (int32_t)p[f], (int32_t)q[f], (int32_t)p[f],
                     (int32_t)(p[f] + q[f])};
            std::copy(st[f].begin(), st[f].end(), hsl.begin() + soff[f]);
        }
        std::vector<int32_t> hrf, hrl, hqf, hql, hpf, hpl;
        std::vector<int64_t> hcp{0}, hci;
        lr_off.assign(1, 0);
        lq_off.assign(1, 0);
        lp_off.assign(1, 0);
        for (int64_t d = 0; d < nlevels; ++d) {
            for (int32_t f : bylev[d]) {
                // children's contributions per local row, in child order
                std::vector<std::vector<int64_t>> contrib(p[f] + q[f]);
                for (int32_t cf : T.ch[f])
                    for (int64_t k = 0; k < q[cf]; ++k) {
                        const int64_t dr = maps[soff[cf] + k];  // dense row -> row list index
                        contrib[dr < pp[f] ? dr : p[f] + (dr - pp[f])].push_back(qoff[cf] + k);
                    }
                for (int64_t r = 0; r < p[f] + q[f]; ++r) {
                    hrf.push_back(f);
                    hrl.push_back((int32_t)r);
                    // a pivot position holds the equation rowp[.] of the front after the exchanges:
                    // its children's contributions follow it
                    const int64_t src = r < p[f] ? rowp[pstart[f] + r] : r;
                    hci.insert(hci.end(), contrib[src].begin(), contrib[src].end());
                    hcp.push_back((int64_t)hci.size());
                }
                for (int64_t k = 0; k < q[f]; ++k) {
                    hqf.push_back(f);
                    hql.push_back((int32_t)k);
                }
                for (int64_t k = 0; k < p[f]; ++k) {
                    hpf.push_back(f);
                    hpl.push_back((int32_t)k);
                }
            }
            lr_off.push_back((int64_t)hrf.size());
            lq_off.push_back((int64_t)hqf.size());
            lp_off.push_back((int64_t)hpf.size());
        }
        auto up = [&](auto &dst, const auto &v) {
            dst.alloc(std::max<size_t>(v.size(), 1));
            if (!v.empty())
                HIPCHK(hipMemcpyAsync(dst.p, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice, c.st));
        };
        up(S, hS);
        up(slist, hsl);
        up(perm, permh);
        up(rperm, rpermh);
        up(rf, hrf);
        up(rl, hrl);
        up(qf, hqf);
        up(ql, hql);
        up(pf, hpf);
        up(pl, hpl);
        up(cptr, hcp);
        up(cidx, hci);
        c.sync();
        Mref = &M;
        // iterative refinement steps (MUMPS's ICNTL(10), default 0): the front
        // inverses (LU-based tile inverses) leave LAPACK-level residuals
        refine = (int)o.integer("pls.lu_refine", 0);
        // perturbed pivots: the factorization is of a nearby matrix; refinement recovers the solve
        if (static_pivots > 0) refine = std::max(refine, (int)o.integer("pls.lu_static_refine", 2));
        if (refine > 0 && !M.sell) build_sell(const_cast<DevCSR &>(M), c);
        setup_s[0] = t1 - t0;
        setup_s[1] = t2 - t1;
        setup_s[2] = t3 - t2;
        setup_s[3] = now_s() - t0;
        // perturbed pivots are reported always (MUMPS reports its own as warnings, INFO(1) > 0;
        // not only under pls.lu_view)
        if (static_pivots > 0 && !o.flag("pls.lu_view", false))
            fprintf(stderr,
                    "[sparse lu] n %lld: %d pivots below %.1e perturbed (static pivoting, pls.lu_static_pivot); "
                    "%d refinement steps per solve\n",
                    (long long)n, static_pivots, tau_used, refine);
        maxf = 0;
        for (int32_t f : post) maxf = std::max(maxf, p[f] + q[f]);
    }

    bool reentrant() const override { return true; }

    // y = M^-1 x with `refine` steps of iterative refinement (y += LU^-1 (x - M y)):
    // the explicit front inverses lose ~cond(F11) eps on ill-conditioned blocks
    // (footing's undrained solid block: 4e-7 relative residual unrefined,
    // rounding level after one step); a fixed number of steps keeps the PC linear.
    void apply(const double *xin, double *y, Ctx &c) override {
        if (n == 0) return;
        auto &w = work[c.st];
        if (!w) w = std::make_unique<DBuf<double>>((size_t)(5 * n + 2 * std::max<int64_t>(nq, 1)));
        double *r = w->p + 3 * n + 2 * std::max<int64_t>(nq, 1), *d = r + n;
        solve(xin, y, *w, c);
        for (int k = 0; k < refine; ++k) {
            spmv(*Mref, y, r, c, -1.0, 1.0, xin);
            solve(r, d, *w, c);
            launch_axpby(n, 1.0, d, 1.0, y, c.st);
        }
    }
    const DevCSR *Mref = nullptr;
    int refine = 1;

    void solve(const double *xin, double *y, DBuf<double> &w, Ctx &c) {
        double *bp = w.p, *z = bp + n, *x = z + n, *cu = x + n, *acc = cu + std::max<int64_t>(nq, 1);
        launch_gather_i32(n, rperm.p, xin, bp, c.st);
        for (int64_t d = nlevels - 1; d >= 0; --d) {
            launch_mf_fwd_gather(lr_off[d + 1] - lr_off[d], rf.p + lr_off[d], rl.p + lr_off[d], S.p,
                                 cptr.p + lr_off[d], cidx.p, bp, cu, z, acc, c.st);
            launch_mf_fwd_gemv(lq_off[d + 1] - lq_off[d], qf.p + lq_off[d], ql.p + lq_off[d], S.p, X.p, z, acc, cu,
                               c.st);
        }
        for (int64_t d = 0; d < nlevels; ++d)
            launch_mf_bwd(lp_off[d + 1] - lp_off[d], pf.p + lp_off[d], pl.p + lp_off[d], S.p, U.p, slist.p, z, x,
                          c.st);
        launch_scatter_i32(n, perm.p, x, y, c.st);
    }
};

std::unique_ptr<PC> make_sparse_lu(const DevCSR &M, const Options &o, Ctx &c) {
    return std::make_unique<PCSparseLU>(M, o, c);
}

}  // namespace pls
