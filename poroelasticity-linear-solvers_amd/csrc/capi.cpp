// capi.cpp -- the handle, the block preconditioner, AAR / Anderson
// acceleration and the extern "C" entry points declared in include/pls.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <numeric>

#include "../../include/pls.h"
#include "runtime.hpp"
#include "amg_host.hpp"

namespace pls {

static thread_local std::string g_last_error;

// ===================================================== synthetic (host) ===
// Offsets per forward block (SURVEY.md 8(d) spec; same definition as the CPU
// oracle so both build the identical matrix).
static inline uint64_t mix64h(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline uint64_t hash3h(uint64_t s, uint64_t a, uint64_t b) { return mix64h(mix64h(mix64h(s) ^ a) ^ b); }

struct SynthHost {
    int dim = 3, N = 1;
    uint64_t seed = 0;
    double delta = 0.05;
    int64_t n[3] = {0, 0, 0}, off[3] = {0, 0, 0}, W[3] = {0, 0, 0};
    int cnt[6] = {0};
    std::vector<int32_t> offs[6];
    void init(const pls_synth_spec &s) {
        dim = s.dim;
        N = s.N;
        seed = s.seed;
        delta = s.delta;
        if (N < 1 || (dim != 2 && dim != 3)) throw Error("synthetic spec: dim must be 2 or 3 and N >= 1");
        const int64_t q = 2 * (int64_t)N + 1, v = (int64_t)N + 1;
        if (dim == 3) {
            n[0] = n[1] = 3 * q * q * q;
            n[2] = v * v * v;
            W[0] = W[1] = 6 * q * q;
            W[2] = v * v + v + 1;
            const int c[6] = {85, 85, 8, 85, 8, 15};
            std::copy(c, c + 6, cnt);
        } else {
            n[0] = n[1] = 2 * q * q;
            n[2] = v * v;
            W[0] = W[1] = 4 * q;
            W[2] = v + 1;
            const int c[6] = {23, 23, 5, 23, 5, 7};
            std::copy(c, c + 6, cnt);
        }
        off[0] = 0;
        off[1] = n[0];
        off[2] = n[0] + n[1];
        if (n[0] + n[1] + n[2] >= (int64_t)INT32_MAX) throw Error("synthetic system too large for int32 columns");
        static const int colf[6] = {0, 1, 2, 1, 2, 2};
        for (int b = 0; b < 6; ++b) {
            const bool sym = (b == 0 || b == 1 || b == 3 || b == 5);
            const int want = cnt[b];
            const int half = sym ? want / 2 : want;
            const int64_t Wb = W[colf[b]];
            const uint64_t range = sym ? (uint64_t)Wb : (uint64_t)(2 * Wb + 1);
            if ((uint64_t)half > range) throw Error("synthetic spec: band too narrow for N");
            uint64_t st = hash3h(seed ^ 0x0FF5E7ULL, (uint64_t)b, 0x51ULL);
            std::vector<int32_t> tmp;
            while ((int)tmp.size() < half) {
                st = mix64h(st);
                const int64_t d = sym ? (int64_t)(1 + st % range) : (int64_t)(st % range) - Wb;
                if (std::find(tmp.begin(), tmp.end(), (int32_t)d) == tmp.end()) tmp.push_back((int32_t)d);
            }
            offs[b].clear();
            if (sym) {
                for (int32_t d : tmp) { offs[b].push_back(d); offs[b].push_back(-d); }
                offs[b].push_back(0);
            } else {
                offs[b] = tmp;
            }
            std::sort(offs[b].begin(), offs[b].end());
        }
    }
    bool is_bc(int64_t ip) const { return (hash3h(seed ^ 0x00BC00ULL, (uint64_t)ip, 7ULL) & 15ULL) == 0ULL; }
};

// ============================================================ Anderson ===
// Least squares min ||f + F a|| for the Anderson steps.  The reference
// (lib/AAR.py:102-105, lib/AndersonAcceleration.py:62-65) gathers F and f to
// rank 0 and runs numpy's Householder QR, then solve(R, -Q^T f).  Here a
// Householder TSQR of the panel [F | f] on the device (k_tsqr: 512-row
// chunks, then the stacked R's, a fixed tree), one m x m R per rank; across
// ranks the R's are all-gathered (m^2 doubles each) and the stack is factored
// on the host in rank order.  The last column of R~ = [[R, z], [0, rho]]
// holds z = Q^T f in R's own sign convention, so a = R^-1 (-z) -- the same
// quantity numpy computes, by a Householder QR, so it stays backward stable up
// to cond(F) ~ 1/eps (no Gram matrix squares the condition number).  Only an
// exactly singular R fails, as numpy.linalg.solve raises LinAlgError.
static void householder_qr_host(std::vector<double> &A, int rows, int m) {  // column-major rows x m, in place
    for (int j = 0; j < m && j < rows; ++j) {
        double sigma = 0.0;
        for (int r = j + 1; r < rows; ++r) sigma += A[(size_t)j * rows + r] * A[(size_t)j * rows + r];
        const double alpha = A[(size_t)j * rows + j];
        if (sigma == 0.0) continue;
        const double nrm = std::sqrt(alpha * alpha + sigma);
        const double beta = alpha >= 0.0 ? -nrm : nrm, tau = (beta - alpha) / beta, scal = 1.0 / (alpha - beta);
        for (int k = j + 1; k < m; ++k) {
            double s = 0.0;
            for (int r = j + 1; r < rows; ++r) s += A[(size_t)j * rows + r] * A[(size_t)k * rows + r];
            const double w = A[(size_t)k * rows + j] + scal * s;
            A[(size_t)k * rows + j] -= tau * w;
            for (int r = j + 1; r < rows; ++r) A[(size_t)k * rows + r] -= tau * w * (A[(size_t)j * rows + r] * scal);
        }
        A[(size_t)j * rows + j] = beta;
    }
}

struct AndersonLS {
    DBuf<const double *> dptr;  // column pointers of every TSQR level
    DBuf<double> lvl[2];        // ping-pong stacks of R's
    DBuf<double> Rdev;          // m x m, then G x m x m gathered
    std::vector<double> solve(const std::vector<const double *> &cols, const double *f, int64_t n, Ctx &c) {
        const int L = (int)cols.size();
        if (L < 1) return {};
        if (L + 1 > 16) throw Error("Anderson order > 15 not supported");
        const int m = L + 1;
        const int64_t C = tsqr_rows_per_block();
        // the TSQR tree: level 0 reads [F | f]; level l > 0 reads level l-1's stacked R's
        std::vector<int64_t> rows{std::max<int64_t>(n, 1)};
        while ((rows.back() + C - 1) / C > 1) rows.push_back(((rows.back() + C - 1) / C) * m);
        const int nlev = (int)rows.size();
        const size_t cap = (size_t)((rows[0] + C - 1) / C) * m * m;
        if (lvl[0].n < cap) { lvl[0].alloc(cap); lvl[1].alloc(cap); }
        if (dptr.n < (size_t)nlev * 16) dptr.alloc((size_t)nlev * 16);
        const int G = c.comm->size;
        if (Rdev.n < (size_t)(G + 1) * m * m) Rdev.alloc((size_t)(G + 1) * m * m);
        std::vector<const double *> hp((size_t)nlev * 16, nullptr);
        for (int k = 0; k < L; ++k) hp[k] = cols[k];
        hp[L] = f;
        for (int l = 1; l < nlev; ++l)
            for (int k = 0; k < m; ++k) hp[(size_t)l * 16 + k] = lvl[(l - 1) & 1].p + (size_t)k * rows[l];
        HIPCHK(hipMemcpyAsync((void *)dptr.p, hp.data(), sizeof(double *) * hp.size(), hipMemcpyHostToDevice, c.st));
        if (n == 0) HIPCHK(hipMemsetAsync(Rdev.p, 0, sizeof(double) * m * m, c.st));  // a rank without rows
        for (int l = 0; l < nlev && n > 0; ++l) {
            const bool last = l == nlev - 1;
            double *out = last ? Rdev.p : lvl[l & 1].p;
            const int64_t ldo = last ? m : ((rows[l] + C - 1) / C) * m;
            launch_tsqr(rows[l], m, dptr.p + (size_t)l * 16, out, ldo, c.st);
        }
        std::vector<double> R((size_t)m * m);
        if (G > 1) {
            double *gat = Rdev.p + (size_t)m * m;
            c.comm->allgather_dev(Rdev.p, m * m, gat, c.st);
            std::vector<double> S((size_t)G * m * m);
            HIPCHK(hipMemcpyAsync(S.data(), gat, sizeof(double) * S.size(), hipMemcpyDeviceToHost, c.st));
            c.sync();
            // stack the ranks' R's in rank order: (G m) x m column-major, then QR
            const int rows_s = G * m;
            std::vector<double> A((size_t)rows_s * m);
            for (int g = 0; g < G; ++g)
                for (int k = 0; k < m; ++k)
                    for (int i = 0; i < m; ++i) A[(size_t)k * rows_s + g * m + i] = S[(size_t)g * m * m + (size_t)k * m + i];
            householder_qr_host(A, rows_s, m);
            for (int k = 0; k < m; ++k)
                for (int i = 0; i < m; ++i) R[(size_t)k * m + i] = i <= k ? A[(size_t)k * rows_s + i] : 0.0;
        } else {
            HIPCHK(hipMemcpyAsync(R.data(), Rdev.p, sizeof(double) * R.size(), hipMemcpyDeviceToHost, c.st));
            c.sync();
        }
        // R~ column-major: R(i, k) = R[k m + i]; z = R~(0:L, L)
        std::vector<double> a(L, 0.0);
        for (int i = L - 1; i >= 0; --i) {
            const double d = R[(size_t)i * m + i];
            if (d == 0.0) throw Error("Anderson least squares: singular R (numpy.linalg.solve raises LinAlgError)");
            double s = -R[(size_t)L * m + i];
            for (int k = i + 1; k < L; ++k) s -= R[(size_t)k * m + i] * a[k];
            a[i] = s / d;
        }
        return a;
    }
};

// y = y + beta * f + sum_{i<mk} alpha_i (X_i + beta F_i)   (AAR.py:109-111)
__global__ void k_anderson_update(int64_t n, int mk, const double *const *X, const double *const *F,
                                  const double *alpha, double beta, const double *f, double *y) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        // the oracle's operation order, no contraction (AAR.py:109-111)
        double v = __dadd_rn(y[e], __dmul_rn(beta, f[e]));
        for (int i = 0; i < mk; ++i) v = __dadd_rn(v, __dmul_rn(alpha[i], __dadd_rn(X[i][e], __dmul_rn(beta, F[i][e]))));
        y[e] = v;
    }
}

struct RingVecs {
    DBuf<double> store;
    int cap = 0;
    int64_t n = 0;
    std::deque<int> live;
    std::vector<int> free_;
    void init(int capacity, int64_t n_) {
        cap = capacity;
        n = n_;
        store.alloc((size_t)std::max(cap, 1) * std::max<int64_t>(n, 1));
        live.clear();
        free_.clear();
        for (int i = cap - 1; i >= 0; --i) free_.push_back(i);
    }
    double *slot(int s) const { return store.p + (int64_t)s * n; }
    // append a copy of v; pop the oldest when more than `keep` remain
    void append(const double *v, int keep, Ctx &c) {
        if (free_.empty()) { free_.push_back(live.front()); live.pop_front(); }
        int s = free_.back();
        free_.pop_back();
        launch_copy(n, v, slot(s), c.st);
        live.push_back(s);
        while ((int)live.size() > keep) { free_.push_back(live.front()); live.pop_front(); }
    }
    int size() const { return (int)live.size(); }
    const double *at(int i) const { return slot(live[i]); }
};

struct AndersonMixer {  // lib/AndersonAcceleration.py:19-78
    int order = 0;
    int64_t k = 0;
    int64_t n = 0;
    DBuf<double> xk, fk, dxk, dfk;
    RingVecs F, X;
    AndersonLS ls;
    DBuf<const double *> pX, pF;
    DBuf<double> dalpha;
    void init(int order_, int64_t n_) {
        order = order_;
        n = n_;
        if (order <= 0) return;
        xk.alloc(n); fk.alloc(n); dxk.alloc(n); dfk.alloc(n);
        F.init(order + 1, n);
        X.init(order + 1, n);
        pX.alloc(16); pF.alloc(16); dalpha.alloc(16);
    }
    void next(double *gk, Ctx &c) {
        if (k == 0) {
            launch_set(n, 0.0, xk.p, c.st);
            launch_set(n, 0.0, fk.p, c.st);
        }
        launch_copy(n, fk.p, dfk.p, c.st);
        launch_copy(n, xk.p, dxk.p, c.st);
        launch_waxpby(n, 1.0, gk, -1.0, xk.p, fk.p, c.st);  // fk = gk - xk
        const int64_t mk = std::min<int64_t>(k, order);
        if (mk > 0) {
            launch_waxpby(n, 1.0, fk.p, -1.0, dfk.p, dfk.p, c.st);  // dfk = fk - dfk
            if (c.norm2(n, dfk.p) < 1e-12) {
                k -= 1;
                launch_copy(n, gk, xk.p, c.st);
            } else {
                F.append(dfk.p, order, c);
                std::vector<const double *> cols;
                for (int i = 0; i < F.size(); ++i) cols.push_back(F.at(i));
                std::vector<double> alpha = ls.solve(cols, fk.p, n, c);
                if ((int64_t)X.size() < mk || (int64_t)F.size() < mk)
                    throw Error("AndersonAcceleration: history shorter than mk (reference raises IndexError)");
                std::vector<const double *> hx, hf;
                for (int64_t i = 0; i < mk; ++i) { hx.push_back(X.at((int)i)); hf.push_back(F.at((int)i)); }
                HIPCHK(hipMemcpyAsync((void *)pX.p, hx.data(), sizeof(double *) * mk, hipMemcpyHostToDevice, c.st));
                HIPCHK(hipMemcpyAsync((void *)pF.p, hf.data(), sizeof(double *) * mk, hipMemcpyHostToDevice, c.st));
                HIPCHK(hipMemcpyAsync(dalpha.p, alpha.data(), sizeof(double) * mk, hipMemcpyHostToDevice, c.st));
                k_anderson_update<<<2048, 256, 0, c.st>>>(n, (int)mk, pX.p, pF.p, dalpha.p, 1.0, fk.p, xk.p);
                c.sync();
            }
        } else {
            launch_copy(n, gk, xk.p, c.st);
        }
        launch_waxpby(n, 1.0, xk.p, -1.0, dxk.p, dxk.p, c.st);  // dxk = xk - dxk
        X.append(dxk.p, order, c);
        k += 1;
        launch_copy(n, xk.p, gk, c.st);
    }
};

// ====================================================== block PC (apply) ===
struct Handle;
struct BlockPC : PC {
    Handle *h = nullptr;
    void apply(const double *x, double *y, Ctx &c) override;
};

// ========================================================== distribution ===
// Row slabs per field (the analogue of PETSc MPIAIJ ownership ranges): rank r
// owns rows [lo_f, lo_f + len_f) of every field f; local layout [s_r | f_r | p_r].
// Synthetic systems use PETSc's split (the first n % size ranks one row
// more); caller matrices (pls_create_dist) bring their own per-rank counts --
// the rows each rank's index sets select, as PETSc's createSubMatrix keeps them.
struct Dist {
    int rank = 0, size = 1;
    int64_t n[3] = {0, 0, 0}, off[3] = {0, 0, 0}, lo[3] = {0, 0, 0}, len[3] = {0, 0, 0}, loff[3] = {0, 0, 0};
    int64_t nloc = 0;
    std::vector<int64_t> start[3];  // start[f][q]: first row of field f owned by rank q (size + 1 entries)
    static void slab(int64_t N, int size, int r, int64_t &lo, int64_t &len) {
        const int64_t q = N / size, rem = N % size;
        lo = r * q + std::min<int64_t>(r, rem);
        len = q + (r < rem ? 1 : 0);
    }
    void range(int f, int q, int64_t &lo_, int64_t &len_) const {
        lo_ = start[f][q];
        len_ = start[f][q + 1] - lo_;
    }
    // counts[f][q] = rows of field f on rank q
    void init_counts(const std::vector<int64_t> counts[3], int r, int s) {
        rank = r;
        size = s;
        int64_t o = 0, lo_ = 0;
        for (int f = 0; f < 3; ++f) {
            start[f].assign(s + 1, 0);
            for (int q = 0; q < s; ++q) start[f][q + 1] = start[f][q] + counts[f][q];
            n[f] = start[f][s];
            off[f] = o;
            o += n[f];
            lo[f] = start[f][r];
            len[f] = counts[f][r];
            loff[f] = lo_;
            lo_ += len[f];
        }
        nloc = lo_;
    }
    void init(const int64_t nf[3], int r, int s) {
        std::vector<int64_t> counts[3];
        for (int f = 0; f < 3; ++f) {
            counts[f].resize(s);
            for (int q = 0; q < s; ++q) {
                int64_t l0, l1;
                slab(nf[f], s, q, l0, l1);
                counts[f][q] = l1;
            }
        }
        init_counts(counts, r, s);
    }
};

// Turn a local-row matrix whose columns are indices into the column space of
// fields [f0, f1] (0 = first column of field f0) into a distributed matrix:
// owned columns -> local index (my slabs of those fields, field order), other
// referenced columns -> ghosts nlocal + position (owner-major, then global),
// plus the halo plan.  Builds the SELL-64 copy.
static void make_dist(DevCSR &M, const Dist &D, int f0, int f1, Comm *comm, Ctx &c) {
    int64_t gsize = 0, nlocal = 0;
    int64_t cs_off[3] = {0, 0, 0}, l_off[3] = {0, 0, 0};
    for (int f = f0; f <= f1; ++f) {
        cs_off[f] = gsize;
        l_off[f] = nlocal;
        gsize += D.n[f];
        nlocal += D.len[f];
    }
    std::vector<int32_t> own(gsize, -1);
    for (int f = f0; f <= f1; ++f)
        for (int64_t i = 0; i < D.len[f]; ++i) own[cs_off[f] + D.lo[f] + i] = (int32_t)(l_off[f] + i);
    DBuf<int32_t> down(std::max<int64_t>(gsize, 1));
    DBuf<uint8_t> dflag(std::max<int64_t>(gsize, 1));
    HIPCHK(hipMemcpyAsync(down.p, own.data(), sizeof(int32_t) * gsize, hipMemcpyHostToDevice, c.st));
    HIPCHK(hipMemsetAsync(dflag.p, 0, gsize, c.st));
    launch_flag_ghosts(M.nnz, M.ci.p, down.p, dflag.p, c.st);
    std::vector<uint8_t> flag(gsize);
    HIPCHK(hipMemcpyAsync(flag.data(), dflag.p, gsize, hipMemcpyDeviceToHost, c.st));
    c.sync();
    std::vector<std::vector<int64_t>> need(D.size);
    std::vector<int32_t> gmap(own);
    int64_t pos = 0;
    auto H = std::make_shared<Halo>();
    H->rcnt.assign(D.size, 0);
    H->roff.assign(D.size, 0);
    for (int q = 0; q < D.size; ++q) {
        H->roff[q] = pos;
        if (q == D.rank) continue;
        for (int f = f0; f <= f1; ++f) {
            int64_t lo, len;
            D.range(f, q, lo, len);
            for (int64_t i = 0; i < len; ++i) {
                const int64_t g = cs_off[f] + lo + i;
                if (flag[g]) {
                    gmap[g] = (int32_t)(nlocal + pos++);
                    need[q].push_back(g);
                }
            }
        }
        H->rcnt[q] = (int64_t)need[q].size();
    }
    H->nlocal = nlocal;
    H->nghost = pos;
    H->l2g.resize(nlocal + pos);
    for (int f = f0; f <= f1; ++f)
        for (int64_t i = 0; i < D.len[f]; ++i) H->l2g[l_off[f] + i] = cs_off[f] + D.lo[f] + i;
    for (int q = 0, k = 0; q < D.size; ++q)
        for (int64_t g : need[q]) H->l2g[nlocal + k++] = g;
    std::vector<std::vector<int64_t>> asked;
    comm->alltoallv_i64(need, asked);
    std::vector<int32_t> sidx;
    H->scnt.assign(D.size, 0);
    H->soff.assign(D.size, 0);
    for (int q = 0; q < D.size; ++q) {
        H->soff[q] = (int64_t)sidx.size();
        for (int64_t g : asked[q]) {
            if (g < 0 || g >= gsize || own[g] < 0) throw Error("halo plan: peer asked for a column this rank does not own");
            sidx.push_back(own[g]);
        }
        H->scnt[q] = (int64_t)asked[q].size();
    }
    H->nsend = (int64_t)sidx.size();
    H->send_idx.alloc(std::max<int64_t>(H->nsend, 1));
    if (H->nsend) HIPCHK(hipMemcpyAsync(H->send_idx.p, sidx.data(), sizeof(int32_t) * H->nsend, hipMemcpyHostToDevice, c.st));
    H->sendbuf.alloc(std::max<int64_t>(H->nsend, 1));
    H->ghost.alloc(std::max<int64_t>(H->nghost, 1));
    DBuf<int32_t> dgmap(std::max<int64_t>(gsize, 1));
    HIPCHK(hipMemcpyAsync(dgmap.p, gmap.data(), sizeof(int32_t) * gsize, hipMemcpyHostToDevice, c.st));
    launch_remap_cols(M.nnz, M.ci.p, dgmap.p, c.st);
    launch_sort_rows(M.nrows, M.rp.p, M.ci.p, M.val.p, c.st);
    HIPCHK(hipGetLastError());
    c.sync();
    M.ncols = nlocal + H->nghost;
    M.halo = H;
    M.sell.reset();
    build_sell(M, c);
}

// ================================================================ handle ===
static void validate_pc_type(const Options &o) {
    std::string pt = o.str("pls.pc_type", "diagonal");
    std::replace(pt.begin(), pt.end(), '_', ' ');
    static const char *ok[] = {"undrained", "undrained 3-way", "diagonal", "diagonal 3-way", "diagonal 3-way-II", "lu"};
    for (auto s : ok)
        if (pt == s) return;
    throw Error("pc type must be one of lu, undrained, diagonal, diagonal 3-way, diagonal 3-way-II.");
}

struct Handle {
    Ctx ctx;
    Options opt;
    Timers timers;
    int64_t n = 0, ns = 0, nf = 0, np = 0;
    bool three_way = false, setup_done = false, solver_ready = false, keep = true;
    Dist dist;                          // row slabs (size 1: everything local)
    bool distributed = false;
    std::unique_ptr<SynthDev> synth_rows;  // synthetic handles: row map for the rhs
    DBuf<int32_t> synth_offs;
    std::string pc_type, solver_type, inner_ksp, inner_pc;
    std::vector<int64_t> perm;   // internal -> caller
    std::vector<int32_t> fp_is_f, fp_is_p;  // 2-way: f / p positions inside the sorted fp set (IndexSet.py:10-26)
    std::unique_ptr<PCFieldSplit> fs_fp;     // fp_ fieldsplit PC (2-way, inexact inner PC)
    std::unique_ptr<PC> pc_red_fp;           // ... on a sharded fp block: gathered, redundant
    bool mixer_ready = false;
    DBuf<int64_t> dperm;
    DevCSR A, P, Pd;
    bool have_Pd = false;
    std::vector<int32_t> bcs;
    DBuf<int32_t> dbcs;
    // sub-blocks (field-major)
    DevCSR Ks, Kf, Kp, Kpd, Kfp, Mfp_s, Ms_fp, Mf_p;
    std::unique_ptr<KSP> ksp_s, ksp_f, ksp_p, ksp_pd, ksp_fp, outer;
    BlockPC bpc;
    AndersonMixer mixer;
    // AAR state (lib/AAR.py)
    struct {
        int order = 10, p = 5;
        double omega = 1.0, beta = 1.0, atol = 1e-8, rtol = 1e-6;
        int64_t maxiter = 500;
        bool monitor = false;
        RingVecs F, X;
        AndersonLS ls;
        DBuf<double> xk, fk, dxk, dfk, tmp;
        DBuf<const double *> pX, pF;
        DBuf<double> dalpha;
        bool init = false;
    } aar;
    // work
    DBuf<double> t_fp, t_s, t_f, xpd, yfpd, ysd, vin, vout;
    DBuf<double> t_s2, t_f2;              // DIFF-sweep temporaries (concurrent 3-way sweeps)
    std::unique_ptr<Ctx> ctx2;            // second stream: the DIFF sweep runs beside the FS sweep
    hipEvent_t ev_in = nullptr, ev_out = nullptr;
    bool concurrent_3way = false;
    // 2-way pressure-first pipeline (pls.fp_pipeline): the fp block's heavy
    // BJACOBI blocks (the pressure rows: ~5x the levels of the fluid blocks)
    // get their t = x_fp - P_fp,s y_s rows first and sweep on the second
    // stream while the fluid rows' product runs (same sums, same blocks)
    struct {
        bool on = false;
        int64_t b_split = 0, nb = 0, r_split = 0, n_hi = 0, n_lo = 0;
        int rr = 0;  // the heavy blocks' sweep: round robin over groups of rr waves (0: every wave per level)
        size_t lds = 0;  // LDS the concurrent product's workgroups reserve (pls.fp_pipeline_lds)
        int tpb = 0, depth = 2;  // the heavy blocks' sweep: threads per workgroup, levels in flight
        bool profiled = false;
        // CU-masked streams (pls.fp_pipeline_cus R > 0): the heavy sweep on R
        // reserved CUs, the concurrent product on the others -- with every CU
        // open to both, the product's workgroups (dispatched first) kept the
        // sweep's from starting until the product drained (measured: the 11
        // sweep workgroups all started ~0.75 ms late)
        std::unique_ptr<Ctx> c_p, c_lo;
        hipEvent_t ev_lo = nullptr;
        int cus = 0;
        DBuf<int32_t> sl_hi, sl_lo;  // Mfp_s slices holding rows >= r_split / the rest
        hipEvent_t ev_t = nullptr, ev_p = nullptr;
    } fpp;
    ~Handle() {
        if (ev_in) (void)hipEventDestroy(ev_in);
        if (ev_out) (void)hipEventDestroy(ev_out);
        if (fpp.ev_t) (void)hipEventDestroy(fpp.ev_t);
        if (fpp.ev_p) (void)hipEventDestroy(fpp.ev_p);
        if (fpp.ev_lo) (void)hipEventDestroy(fpp.ev_lo);
    }
    // result
    pls_result res{};
    std::vector<double> history;
    int pc_applies = 0;
    std::unique_ptr<MatOp> Aop;

    void parse_params() {
        pc_type = opt.str("pls.pc_type", "diagonal");
        static const char *ok[] = {"undrained", "undrained 3-way", "diagonal", "diagonal 3-way", "diagonal 3-way-II",
                                   "lu"};
        // values with spaces are passed with '_' or as the literal tail
        std::string pt = pc_type;
        std::replace(pt.begin(), pt.end(), '_', ' ');
        pc_type = pt;
        bool good = false;
        for (auto s : ok) good = good || (pc_type == s);
        if (!good) throw Error("pc type must be one of lu, undrained, diagonal, diagonal 3-way, diagonal 3-way-II.");
        three_way = (pc_type == "diagonal 3-way" || pc_type == "undrained 3-way");
        solver_type = opt.str("pls.solver_type", "gmres");
        inner_ksp = opt.str("pls.inner_ksp_type", "gmres");
        inner_pc = opt.str("pls.inner_pc_type", "hypre");
        timers.enabled = opt.flag("pls.timers", true);
        ctx.sell_d16 = opt.flag("pls.sell_d16", true);
        ctx.d16_wide_lpr = (int)opt.integer("pls.d16_wide_lpr", 8);
        if (ctx.d16_wide_lpr != 1 && ctx.d16_wide_lpr != 2 && ctx.d16_wide_lpr != 4 && ctx.d16_wide_lpr != 8 &&
            ctx.d16_wide_lpr != 16 && ctx.d16_wide_lpr != 32 && ctx.d16_wide_lpr != 64)
            throw Error("pls.d16_wide_lpr must be a power of two <= 64");
        ctx.d16_unroll = (int)opt.integer("pls.d16_unroll", 4);
        ctx.halo_overlap = opt.flag("pls.halo_overlap", true);
        ctx.d16_segs = (int)opt.integer("pls.d16_segs", D16_SEG);  // 8: force the halo layout (tests)
        if (ctx.d16_segs != D16_SEG && ctx.d16_segs != D16_SEG_MAX) throw Error("pls.d16_segs must be 4 or 8");
        set_d16_xcd((int)opt.integer("pls.d16_xcd", 0));  // process-wide (tuning)
        set_spmv_short_rows(opt.flag("pls.spmv_short", false));  // process-wide (measured slower for the AMG's P)
        if (opt.integer("pls.ilu0_probe", 0)) set_ilu0_probe((int)opt.integer("pls.ilu0_probe", 0));  // diagnostics
        set_ring_probe((int)opt.integer("pls.ring_probe", 0));  // diagnostics (every handle: its own setting)
        ctx.d16_sigma = (int)opt.integer("pls.d16_sigma", 1024);
        if (ctx.d16_sigma < 0 || ctx.d16_sigma % 64) throw Error("pls.d16_sigma must be a multiple of 64 (0: off)");
        ctx.d16_sigma_pad = opt.num("pls.d16_sigma_pad", 0.15);
        ctx.d16_sorted_lpr = (int)opt.integer("pls.d16_sorted_lpr", 2);
        ctx.spmv_b3 = opt.flag("pls.spmv_b3", false);
        ctx.spmv_rcm = (int)opt.integer("pls.spmv_rcm", -1);
        ctx.sweep_chain = (int)opt.integer("pls.sweep_chain", -1);
        ctx.sweep_window = (int)opt.integer("pls.sweep_window", -1);
        ctx.ilu_factor_dep = (int)opt.integer("pls.ilu_factor_dep", 1);
        ctx.ilu_view = (int)opt.integer("pls.ilu_view", 0);
        // test knobs of the ILU(0) factorization: staged-entry cap, persistent grid cap
        ctx.ilu0_stage_cap = (int)opt.integer("pls.ilu0_stage", -1);
        ctx.ilu_dep_grid = (int)opt.integer("pls.ilu_dep_grid", 0);
        ctx.window_depth = (int)opt.integer("pls.window_depth", 2);
        if (ctx.window_depth != 2 && ctx.window_depth != 3) throw Error("pls.window_depth must be 2 or 3");
        ctx.window_ring = (int)opt.integer("pls.window_ring", -1);
        ctx.window_mixed = (int)opt.integer("pls.window_mixed", -1);
        ctx.window_kpw = (int)opt.integer("pls.window_kpw", 0);
        ctx.sweep_swin = (int)opt.integer("pls.sweep_swin", 0);
        ctx.amg_csr_below = opt.num("pls.amg_csr_below", 16.0);
        if (opt.flag("pls.debug_bounds", false) || opt.integer("pls.debug_partial_cap", 0) > 0)
            ctx.set_debug(opt.flag("pls.debug_bounds", false), opt.integer("pls.debug_partial_cap", 0),
                          opt.flag("pls.debug_no_grow", false), opt.flag("pls.debug_unguarded", false));
        if (ctx.d16_sorted_lpr != 1 && ctx.d16_sorted_lpr != 2 && ctx.d16_sorted_lpr != 4 && ctx.d16_sorted_lpr != 8 &&
            ctx.d16_sorted_lpr != 16)
            throw Error("pls.d16_sorted_lpr must be 1, 2, 4, 8 or 16");
    }
};

void BlockPC::apply(const double *x, double *y, Ctx &c) {
    Handle &H = *h;
    Timers &T = H.timers;
    T.begin(T_PC_TOTAL);
    const int64_t ns = H.ns, nf = H.nf, np = H.np;
    if (!H.three_way) {
        T.begin(T_PC_SOLID);
        H.ksp_s->solve(x, y, c);
        T.end(T_PC_SOLID);
        T.begin(T_PC_FLUID);
        if (H.fpp.on) {
            // the heavy blocks' rows of t first, their sweep on the second stream
            // while the other rows' product and sweep run here (a PREONLY solve)
            auto &F = H.fpp;
            Ctx &c2 = F.c_p ? *F.c_p : *H.ctx2;
            Ctx &clo = F.c_lo ? *F.c_lo : c;
            PCILU *pc = static_cast<PCILU *>(H.ksp_fp->pc);
            // pls.ilu_view 3: per-block start / end of both launches, once (diagnostics)
            DBuf<int64_t> prof;
            if (H.ctx.ilu_view >= 3 && !F.profiled) prof.alloc(F.nb * 8);
            spmv_slices(H.Mfp_s, y, H.t_fp.p, c, -1.0, 1.0, x + ns, F.sl_hi.p, F.n_hi);
            HIPCHK(hipEventRecord(F.ev_t, c.st));
            HIPCHK(hipStreamWaitEvent(c2.st, F.ev_t, 0));
            pc->apply_blocks(H.t_fp.p, y + ns, c2, F.b_split, F.nb, F.rr, F.tpb, F.depth, prof.p);
            HIPCHK(hipEventRecord(F.ev_p, c2.st));
            if (F.c_lo) HIPCHK(hipStreamWaitEvent(clo.st, F.ev_t, 0));
            // (pls.fp_pipeline_lds: its workgroups reserve LDS they do not use)
            spmv_slices(H.Mfp_s, y, H.t_fp.p, clo, -1.0, 1.0, x + ns, F.sl_lo.p, F.n_lo, F.lds);
            if (F.c_lo) {
                HIPCHK(hipEventRecord(F.ev_lo, clo.st));
                HIPCHK(hipStreamWaitEvent(c.st, F.ev_lo, 0));
            }
            pc->apply_blocks(H.t_fp.p, y + ns, c, 0, F.b_split, 0, 0, 2, prof.p);
            HIPCHK(hipStreamWaitEvent(c.st, F.ev_p, 0));
            if (prof.p) {
                F.profiled = true;
                std::vector<int64_t> hp(F.nb * 8);
                HIPCHK(hipMemcpyAsync(hp.data(), prof.p, sizeof(int64_t) * hp.size(), hipMemcpyDeviceToHost, c.st));
                c.sync();
                int64_t t0 = INT64_MAX;
                for (int64_t b = 0; b < F.nb; ++b) t0 = std::min(t0, hp[b * 8]);
                auto span = [&](int64_t b0, int64_t b1, const char *what) {
                    int64_t s0 = INT64_MAX, s1 = 0, e1 = 0;
                    double dsum = 0;
                    for (int64_t b = b0; b < b1; ++b) {
                        s0 = std::min(s0, hp[b * 8]);
                        s1 = std::max(s1, hp[b * 8]);
                        e1 = std::max(e1, hp[b * 8 + 2]);
                        dsum += (hp[b * 8 + 2] - hp[b * 8]) * 0.01;
                    }
                    fprintf(stderr, "[pls fp pipeline] %s blocks [%lld, %lld): starts %+.1f .. %+.1f us, last end %+.1f us, "
                            "mean duration %.1f us\n", what, (long long)b0, (long long)b1, (s0 - t0) * 0.01,
                            (s1 - t0) * 0.01, (e1 - t0) * 0.01, dsum / std::max<int64_t>(1, b1 - b0));
                };
                span(F.b_split, F.nb, "heavy");
                span(0, F.b_split, "light");
            }
            H.ksp_fp->note_preonly();
            c.check_bounds();  // (what KSP::solve does after a solve; pls.debug_bounds)
        } else {
            // t = x_fp - P_fp,s y_s   (Preconditioner.py:232-233, fused)
            spmv(H.Mfp_s, y, H.t_fp.p, c, -1.0, 1.0, x + ns);
            H.ksp_fp->solve(H.t_fp.p, y + ns, c);
        }
        T.end(T_PC_FLUID);
    } else {
        const double *xs = x, *xf = x + ns, *xp = x + ns + nf;
        double *ys = y, *yf = y + ns, *yp = y + ns + nf;
        double *yfd = H.yfpd.p, *ypd = H.yfpd.p + nf;
        if (H.concurrent_3way) {
            // FS sweep on the main stream, DIFF sweep on the second; join before the combination
            Ctx &c2 = *H.ctx2;
            HIPCHK(hipEventRecord(H.ev_in, c.st));
            HIPCHK(hipStreamWaitEvent(c2.st, H.ev_in, 0));
            launch_copy(np, xp, H.xpd.p, c2.st);                     // :172-173 BC rows of x_p zeroed
            launch_zero_entries((int64_t)H.bcs.size(), H.dbcs.p, H.xpd.p, c2.st);
            H.ksp_pd->solve(H.xpd.p, ypd, c2);                       // :174
            spmv(H.Mf_p, ypd, H.t_f2.p, c2, -1.0, 1.0, xf);          // :184-185
            H.ksp_f->solve(H.t_f2.p, yfd, c2);                       // :186
            spmv(H.Ms_fp, yfd, H.t_s2.p, c2, -1.0, 1.0, xs);         // :198-201
            H.ksp_s->solve(H.t_s2.p, H.ysd.p, c2);                   // :202
            HIPCHK(hipEventRecord(H.ev_out, c2.st));
            T.begin(T_PC_PRESS);
            H.ksp_p->solve(xp, yp, c);                               // :170
            T.end(T_PC_PRESS);
            T.begin(T_PC_FLUID);
            spmv(H.Mf_p, yp, H.t_f.p, c, -1.0, 1.0, xf);             // :180-181
            H.ksp_f->solve(H.t_f.p, yf, c);                          // :182
            T.end(T_PC_FLUID);
            T.begin(T_PC_SOLID);
            spmv(H.Ms_fp, yf, H.t_s.p, c, -1.0, 1.0, xs);            // :192-195
            H.ksp_s->solve(H.t_s.p, ys, c);                          // :196
            T.end(T_PC_SOLID);
            HIPCHK(hipStreamWaitEvent(c.st, H.ev_out, 0));
            launch_axpby(ns, 0.1, H.ysd.p, 1.0, ys, c.st);           // :207-212
            launch_axpby(nf + np, 0.1, yfd, 1.0, yf, c.st);
            if (H.mixer.order > 0) H.mixer.next(y, c);               // :248-249
            T.end(T_PC_TOTAL);
            H.pc_applies++;
            return;
        }
        T.begin(T_PC_PRESS);
        H.ksp_p->solve(xp, yp, c);                               // :170
        launch_copy(np, xp, H.xpd.p, c.st);                      // :172-173 BC rows of x_p zeroed
        launch_zero_entries((int64_t)H.bcs.size(), H.dbcs.p, H.xpd.p, c.st);
        H.ksp_pd->solve(H.xpd.p, ypd, c);                        // :174
        T.end(T_PC_PRESS);
        T.begin(T_PC_FLUID);
        spmv(H.Mf_p, yp, H.t_f.p, c, -1.0, 1.0, xf);             // :180-181
        H.ksp_f->solve(H.t_f.p, yf, c);                          // :182
        spmv(H.Mf_p, ypd, H.t_f.p, c, -1.0, 1.0, xf);            // :184-185
        H.ksp_f->solve(H.t_f.p, yfd, c);                         // :186
        T.end(T_PC_FLUID);
        T.begin(T_PC_SOLID);
        spmv(H.Ms_fp, yf, H.t_s.p, c, -1.0, 1.0, xs);            // :192-195 (y_f, y_p contiguous)
        H.ksp_s->solve(H.t_s.p, ys, c);                          // :196
        spmv(H.Ms_fp, yfd, H.t_s.p, c, -1.0, 1.0, xs);           // :198-201
        H.ksp_s->solve(H.t_s.p, H.ysd.p, c);                     // :202
        T.end(T_PC_SOLID);
        // y = w1 y_FS + w2 y_DIFF (:207-212)
        launch_axpby(ns, 0.1, H.ysd.p, 1.0, ys, c.st);
        launch_axpby(nf + np, 0.1, yfd, 1.0, yf, c.st);
    }
    if (H.mixer.order > 0) H.mixer.next(y, c);                 // :248-249
    T.end(T_PC_TOTAL);
    H.pc_applies++;
}

// ------------------------------------------------------------ setup path ---
// rows permuted and re-sorted into the internal field order; rows on host
// threads (the footing N=128 system's three 68.8M-entry matrices took ~8 s of
// pls_create on one thread)
static void permute_host(const pls_csr *M, const std::vector<int64_t> &perm, const std::vector<int64_t> &inv,
                         hvec<int64_t> &rp, hvec<int32_t> &ci, hvec<double> &v) {
    const int64_t n = (int64_t)perm.size();
    rp.assign(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) rp[i + 1] = rp[i] + (M->row_ptr[perm[i] + 1] - M->row_ptr[perm[i]]);
    ci.resize(rp[n]);
    v.resize(rp[n]);
    std::atomic<bool> bad{false};
    amgh::parallel_rows(n, amgh::setup_threads(), [&](int, int64_t i0, int64_t i1) {
        std::vector<std::pair<int32_t, double>> row;
        for (int64_t i = i0; i < i1; ++i) {
            const int64_t o = perm[i];
            row.clear();
            for (int64_t k = M->row_ptr[o]; k < M->row_ptr[o + 1]; ++k) {
                const int32_t cc = M->col[k];
                if (cc < 0 || cc >= n) {
                    bad = true;
                    row.emplace_back(0, 0.0);
                    continue;
                }
                row.emplace_back((int32_t)inv[cc], M->val[k]);
            }
            std::sort(row.begin(), row.end(), [](auto &a, auto &b) { return a.first < b.first; });
            for (size_t t = 0; t < row.size(); ++t) {
                ci[rp[i] + t] = row[t].first;
                v[rp[i] + t] = row[t].second;
            }
        }
    });
    if (bad) throw Error("column index out of range");
}

static void upload_permuted(const pls_csr *M, Handle &H, const std::vector<int64_t> &inv, DevCSR &out) {
    if (M->nrows != H.n || M->ncols != H.n) throw Error("matrix must be n x n with n = ns + nf + np");
    hvec<int64_t> rp;
    hvec<int32_t> ci;
    hvec<double> v;
    permute_host(M, H.perm, inv, rp, ci, v);
    upload_csr(out, H.n, H.n, rp.data(), ci.data(), v.data(), H.ctx);
}

// The 2-way PC's fp solve with PREONLY + BJACOBI(ILU(0)) on the LDS sweep:
// when the last blocks (the pressure rows of the field-major fp block) carry
// well over the median block's levels, their rows of t = x_fp - P_fp,s y_s are
// computed first and swept on a second stream beside the rest of the product
// (the headline N=59: 11 pressure blocks of 263 levels per triangle, ~500 us,
// against 56 for the fluid blocks).  Results are bitwise those of the plain
// path: the same per-row sums and per-block sweeps.  pls.fp_pipeline 0 turns
// it off.
static void setup_fp_pipeline(Handle &H) {
    auto &F = H.fpp;
    F.on = false;
    // pls.fp_pipeline: 1 always, 0 never, -1 (default) when the s block's PC is an
    // ILU / BJACOBI sweep too.  Measured (MI355X, N=59, same box, A/B x 3): the
    // BJACOBI headline 168.4 -> 169.8 it/s; with BoomerAMG on the s block 120 ->
    // 114 it/s -- with the CU-masked queues present every kernel of the V-cycle's
    // ~40 per iteration ran slower (small ones ~2-10x), which the pipeline's
    // ~90 us per iteration does not repay
    const int64_t mode = H.opt.integer("pls.fp_pipeline", -1);
    if (H.three_way || H.distributed || mode == 0) return;
    if (!H.ksp_fp || H.ksp_fp->type != "preonly" || H.mixer.order > 0) return;
    if (H.ksp_fp->monitor) return;  // -fp_ksp_monitor: the plain path's KSP::solve prints it
    if (mode < 0 && !(H.ksp_s && H.ksp_s->type == "preonly" && dynamic_cast<PCILU *>(H.ksp_s->pc))) return;
    PCILU *pc = dynamic_cast<PCILU *>(H.ksp_fp->pc);
    if (!pc || !pc->can_apply_blocks() || pc->nblocks < 8 || pc->block_levels_h.size() != (size_t)pc->nblocks) return;
    const DevCSR &M = H.Mfp_s;
    if (!M.sell || !M.sell->d16 || M.halo || M.sell->nperm || M.sell->b3_nslices || M.sell->nrows_mapped) return;
    const int64_t nb = pc->nblocks;
    std::vector<int64_t> lev(pc->block_levels_h);
    std::vector<int64_t> srt(lev);
    std::nth_element(srt.begin(), srt.begin() + nb / 2, srt.end());
    const int64_t med = srt[nb / 2];
    int64_t b = nb;
    while (b > 0 && lev[b - 1] >= 2 * med) --b;
    if (b == nb || nb - b > nb / 8 || b == 0) return;  // no heavy tail, or too much of the block
    const DevSELL &S = *M.sell;
    std::vector<int64_t> sf(S.nslices + 1);
    HIPCHK(hipMemcpyAsync(sf.data(), S.sfirst.p, sizeof(int64_t) * sf.size(), hipMemcpyDeviceToHost, H.ctx.st));
    H.ctx.sync();
    const int64_t r_split = pc->block_start_h[b];
    std::vector<int32_t> hi, lo;
    for (int64_t s = 0; s < S.nslices; ++s) (sf[s + 1] > r_split ? hi : lo).push_back((int32_t)s);
    F.sl_hi.alloc(std::max<size_t>(hi.size(), 1));
    F.sl_lo.alloc(std::max<size_t>(lo.size(), 1));
    if (!hi.empty())
        HIPCHK(hipMemcpyAsync(F.sl_hi.p, hi.data(), sizeof(int32_t) * hi.size(), hipMemcpyHostToDevice, H.ctx.st));
    if (!lo.empty())
        HIPCHK(hipMemcpyAsync(F.sl_lo.p, lo.data(), sizeof(int32_t) * lo.size(), hipMemcpyHostToDevice, H.ctx.st));
    H.ctx.sync();
    if (!H.ctx2) H.ctx2 = std::make_unique<Ctx>();
    if (!F.ev_t) HIPCHK(hipEventCreateWithFlags(&F.ev_t, hipEventDisableTiming));
    if (!F.ev_p) HIPCHK(hipEventCreateWithFlags(&F.ev_p, hipEventDisableTiming));
    // Experimental variants for the heavy sweep (both measured no faster, kept
    // opt-in): round-robin wave groups owning whole levels
    // (pls.fp_pipeline_rr g) and 6 levels of factor data in flight on 8 waves
    // (pls.fp_pipeline_depth 6, levels of <= 8 slices) -- meant for the
    // concurrent product's HBM traffic, which stretches a load's latency past
    // the plain sweep's two levels (the 11 pressure blocks: 1.24 ms beside the
    // unmasked product, ~0.5 ms alone)
    int64_t msl = 0;
    for (int64_t k = b; k < nb; ++k) msl = std::max(msl, pc->block_maxsl_h.empty() ? 16 : pc->block_maxsl_h[k]);
    // pls.fp_pipeline_rr (experimental, measured no faster): 0 / -1 off (default), or a forced group size
    const int64_t rr_opt = H.opt.integer("pls.fp_pipeline_rr", 0);
    if (rr_opt > 16 || (rr_opt > 0 && (rr_opt & (rr_opt - 1))))
        throw Error("pls.fp_pipeline_rr must be 0 (off) or a power of two <= 16");
    const bool deep = msl <= 8 && H.opt.integer("pls.fp_pipeline_depth", 2) == 6;
    F.rr = rr_opt > 0 ? (int)rr_opt : 0;
    F.tpb = deep && F.rr == 0 ? 512 : 0;
    F.depth = deep && F.rr == 0 ? 6 : 2;
    // the sweep holds max_len * 8 bytes of the CU's 160 KiB: reserve more than what is left
    const int64_t left = 163840 - pc->max_len * 8;
    const int64_t lds_opt = H.opt.integer("pls.fp_pipeline_lds", 0);
    F.lds = (size_t)(lds_opt >= 0 ? lds_opt : (left < 16384 ? ((left + 1024) & ~int64_t(1023)) : 0));
    // reserved CUs: the heavy blocks' count rounded up to a multiple of 8 (one per XCD)
    int ncu = 0, dev = 0;
    HIPCHK(hipGetDevice(&dev));
    HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const int64_t cus_opt = H.opt.integer("pls.fp_pipeline_cus", -1);
    const int want = (int)(cus_opt >= 0 ? cus_opt : (nb - b + 7) / 8 * 8);
    F.cus = (want >= nb - b && want <= ncu / 4) ? want : 0;
    F.c_p.reset();
    F.c_lo.reset();
    if (F.cus > 0) {
        const uint32_t words = (uint32_t)((ncu + 31) / 32);
        std::vector<uint32_t> mp(words, 0), ml(words, 0);
        // which mask bits: pls.fp_pipeline_cu_layout 0 -- bits [0, R) (one per XCD in turn
        // if the driver deals bits round robin over the XCDs), 1 -- R / 8 consecutive
        // bits at the start of every 1/8 of the mask (XCD-major bit order)
        const int64_t layout = H.opt.integer("pls.fp_pipeline_cu_layout", 0);
        for (int k = 0; k < ncu; ++k) {
            const int per = ncu / 8;
            const bool res = layout == 1 ? (k % per) < F.cus / 8 : k < F.cus;
            (res ? mp : ml)[k / 32] |= 1u << (k % 32);
        }
        // (a driver without CU masking: plain streams, F.cus = 0)
        auto masked = [&](const std::vector<uint32_t> &m) -> std::unique_ptr<Ctx> {
            auto cx = std::make_unique<Ctx>();
            hipStream_t s = nullptr;
            if (hipExtStreamCreateWithCUMask(&s, words, m.data()) != hipSuccess) {
                (void)hipGetLastError();
                return nullptr;
            }
            HIPCHK(hipStreamDestroy(cx->st));
            cx->st = s;
            cx->d16_unroll = H.ctx.d16_unroll;
            return cx;
        };
        F.c_p = masked(mp);
        F.c_lo = F.c_p ? masked(ml) : nullptr;
        if (!F.c_p || !F.c_lo) {
            F.c_p.reset();
            F.c_lo.reset();
            F.cus = 0;
        }
        if (!F.ev_lo) HIPCHK(hipEventCreateWithFlags(&F.ev_lo, hipEventDisableTiming));
    }
    F.b_split = b;
    F.nb = nb;
    F.r_split = r_split;
    F.n_hi = (int64_t)hi.size();
    F.n_lo = (int64_t)lo.size();
    F.on = true;
    if (H.ctx.ilu_view)
        fprintf(stderr, "[pls fp pipeline] blocks [%lld, %lld) first (levels >= %lld, median %lld), rows from %lld, "
                "slices %lld + %lld, round-robin groups %d (most slices per level %lld), product LDS reserve %zu, "
                "sweep tpb %d depth %d, reserved CUs %d\n", (long long)b, (long long)nb,
                (long long)(2 * med), (long long)med, (long long)r_split, (long long)F.n_hi, (long long)F.n_lo, F.rr,
                (long long)msl, F.lds, F.tpb, F.depth, F.cus);
}

static void alloc_work(Handle &H) {
    H.t_fp.alloc(std::max<int64_t>(H.nf + H.np, 1));
    H.t_s.alloc(std::max<int64_t>(H.ns, 1));
    H.t_f.alloc(std::max<int64_t>(H.nf, 1));
    H.xpd.alloc(std::max<int64_t>(H.np, 1));
    H.yfpd.alloc(std::max<int64_t>(H.nf + H.np, 1));
    H.ysd.alloc(std::max<int64_t>(H.ns, 1));
    H.vin.alloc(std::max<int64_t>(H.n, 1));
    H.vout.alloc(std::max<int64_t>(H.n, 1));
    // 3-way: the FS (p -> f -> s) and DIFF sweeps are independent until the
    // final w1/w2 combination (Preconditioner.py:150-212); with PREONLY inner
    // solves (no host round trips) the DIFF sweep runs on a second stream.
    // Not with several ranks: two streams would interleave halo exchanges on
    // one communicator.
    H.concurrent_3way = false;
    if (H.three_way && !H.distributed && H.opt.flag("pls.concurrent_sweeps", true)) {
        bool pre = true;
        for (KSP *k : {H.ksp_s.get(), H.ksp_f.get(), H.ksp_p.get(), H.ksp_pd.get()}) pre = pre && k && k->type == "preonly";
        // the s and f PCs serve both sweeps at once: they must be reentrant
        for (KSP *k : {H.ksp_s.get(), H.ksp_f.get()}) pre = pre && k->pc && k->pc->reentrant();
        if (pre) {
            if (!H.ctx2) {
                H.ctx2 = std::make_unique<Ctx>();
                HIPCHK(hipEventCreateWithFlags(&H.ev_in, hipEventDisableTiming));
                HIPCHK(hipEventCreateWithFlags(&H.ev_out, hipEventDisableTiming));
            }
            H.t_s2.alloc(std::max<int64_t>(H.ns, 1));
            H.t_f2.alloc(std::max<int64_t>(H.nf, 1));
            H.concurrent_3way = true;
        }
    }
    setup_fp_pipeline(H);
}

static void do_setup(Handle &H) {
    if (H.setup_done) return;
    Ctx &c = H.ctx;
    const int64_t ns = H.ns, nf = H.nf, n = H.n;
    WindowSpec w{};
    w.mode = 0;
    auto ext = [&](const DevCSR &M, int64_t r0, int64_t r1, int64_t c0, int64_t c1, DevCSR &dst) {
        WindowSpec ww{};
        ww.mode = 0;
        ww.c0 = c0;
        ww.c1 = c1;
        extract_csr(M, r0, r1, ww, c0, c1 - c0, dst, c);
    };
    (void)w;
    // lib/Preconditioner.py:60-75 allocate_submatrices (field-major: contiguous ranges)
    if (H.distributed) {
        // local rows, global columns of the fields [f0, f1] -> distributed block
        const Dist &D = H.dist;
        auto dext = [&](const DevCSR &M, int64_t r0, int64_t r1, int f0, int f1, DevCSR &dst) {
            const int64_t g0 = D.off[f0], g1 = D.off[f1] + D.n[f1];
            WindowSpec ww{};
            ww.mode = 0;
            ww.c0 = g0;
            ww.c1 = g1;
            extract_csr(M, r0, r1, ww, g0, g1 - g0, dst, c);
            make_dist(dst, D, f0, f1, c.comm, c);
        };
        const int64_t nfl = H.nf;
        dext(H.P, 0, ns, 0, 0, H.Ks);
        if (!H.three_way) {
            dext(H.P, ns, n, 0, 0, H.Mfp_s);
            dext(H.P, ns, n, 1, 2, H.Kfp);
        } else {
            if (!H.have_Pd) throw Error("3-way preconditioner needs P_diff");
            dext(H.P, ns, ns + nfl, 1, 1, H.Kf);
            dext(H.P, ns + nfl, n, 2, 2, H.Kp);
            dext(H.Pd, ns + nfl, n, 2, 2, H.Kpd);
            dext(H.P, 0, ns, 1, 2, H.Ms_fp);
            dext(H.P, ns, ns + nfl, 2, 2, H.Mf_p);
        }
    } else {
    ext(H.P, 0, ns, 0, ns, H.Ks);
    if (!H.three_way) {
        ext(H.P, ns, n, 0, ns, H.Mfp_s);
        ext(H.P, ns, n, ns, n, H.Kfp);
    } else {
        if (!H.have_Pd) throw Error("3-way preconditioner needs P_diff");
        ext(H.P, ns, ns + nf, ns, ns + nf, H.Kf);
        ext(H.P, ns + nf, n, ns + nf, n, H.Kp);
        ext(H.Pd, ns + nf, n, ns + nf, n, H.Kpd);
        ext(H.P, 0, ns, ns, n, H.Ms_fp);
        ext(H.P, ns, ns + nf, ns + nf, n, H.Mf_p);
    }
    }
    // SELL-64 copies of every matrix the PC multiplies with
    if (!H.three_way) {
        build_sell(H.Mfp_s, c);
    } else {
        build_sell(H.Ms_fp, c);
        build_sell(H.Mf_p, c);
    }
    // (PLS_SETUP_TRACE: wall time of the setup stages on stderr)
    const bool trace = std::getenv("PLS_SETUP_TRACE") != nullptr;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    c.sync();
    double t0 = now();
    auto stage = [&](const char *what) {
        if (!trace) return;
        c.sync();
        const double t1 = now();
        fprintf(stderr, "[setup] %s %.2f s\n", what, t1 - t0);
        t0 = t1;
    };
    stage("blocks extracted");
    // inner solvers (setup_elliptic_solver / setup_fieldsplit; options win)
    const Options &o = H.opt;
    H.ksp_s = make_ksp("s_", o, &H.Ks, &H.Ks, H.inner_ksp, H.inner_pc, c);
    stage("s block solver");
    if (H.three_way) {
        H.ksp_f = make_ksp("f_", o, &H.Kf, &H.Kf, H.inner_ksp, H.inner_pc, c);
        H.ksp_p = make_ksp("p_", o, &H.Kp, &H.Kp, H.inner_ksp, H.inner_pc, c);
        H.ksp_pd = make_ksp("diff_", o, &H.Kpd, &H.Kpd, H.inner_ksp, H.inner_pc, c);
    } else {
        if (H.inner_pc == "lu") {
            H.ksp_fp = make_ksp("fp_", o, &H.Kfp, &H.Kfp, H.inner_ksp, "lu", c);
        } else {
            const std::string pt = o.str("fp_pc_type", "fieldsplit");
            if (pt == "fieldsplit") {
                // setup_fieldsplit (Preconditioner.py:102-118): setFieldSplitIS((None, is_p)) then
                // ((None, is_f)) -- split 0 = pressure, split 1 = fluid, fp-local positions
                if (H.distributed) {
                    // sharded fp block: the fieldsplit PC on the gathered block, redundantly.
                    // Gathered order = the block's global order: synthetic shards are
                    // field-major (split 0 = p = [nf, nf + np), split 1 = f = [0, nf));
                    // caller-assembled ones (pls_create_dist, 2-way: one fp field) are
                    // rank-major, each rank's rows its sorted f U p (PETSc's is_fp), so the
                    // splits are every rank's fp_is_p / fp_is_f offset by its first row
                    std::vector<int32_t> gf, gp;
                    const Dist &D = H.dist;
                    if (D.n[2] == 0) {
                        Comm *cm = c.comm;
                        const int G = cm->size;
                        int64_t mine[2] = {(int64_t)H.fp_is_f.size(), (int64_t)H.fp_is_p.size()};
                        std::vector<int64_t> cnts((size_t)2 * G);
                        cm->allgather_host(mine, sizeof(mine), cnts.data());
                        int64_t mx = 1;
                        for (int64_t v : cnts) mx = std::max(mx, v);
                        std::vector<int32_t> sendf(mx, -1), sendp(mx, -1), allf((size_t)mx * G), allp((size_t)mx * G);
                        std::copy(H.fp_is_f.begin(), H.fp_is_f.end(), sendf.begin());
                        std::copy(H.fp_is_p.begin(), H.fp_is_p.end(), sendp.begin());
                        cm->allgather_host(sendf.data(), sizeof(int32_t) * mx, allf.data());
                        cm->allgather_host(sendp.data(), sizeof(int32_t) * mx, allp.data());
                        for (int q = 0; q < G; ++q) {
                            const int64_t base = D.start[1][q];
                            for (int64_t k = 0; k < cnts[2 * q]; ++k) gf.push_back((int32_t)(base + allf[(size_t)q * mx + k]));
                            for (int64_t k = 0; k < cnts[2 * q + 1]; ++k) gp.push_back((int32_t)(base + allp[(size_t)q * mx + k]));
                        }
                    } else {
                        for (int64_t i = 0; i < D.n[1]; ++i) gf.push_back((int32_t)i);
                        for (int64_t i = 0; i < D.n[2]; ++i) gp.push_back((int32_t)(D.n[1] + i));
                    }
                    H.pc_red_fp = make_redundant("fieldsplit", H.Kfp, c, [&](const DevCSR &Gm, Ctx &sc) -> std::unique_ptr<PC> {
                        return std::make_unique<PCFieldSplit>(Gm, gp, gf, o, "fp_", sc);
                    }, "fp_");
                    H.ksp_fp = make_ksp("fp_", o, &H.Kfp, &H.Kfp, "gmres", "fieldsplit", c, 1e-5, 1e-50, 1e4, 10000, 30,
                                        H.pc_red_fp.get());
                    goto fp_done;
                }
                std::vector<int32_t> fpf = H.fp_is_f, fpp = H.fp_is_p;
                if (fpf.empty() && fpp.empty()) {  // field-major fp block: [f | p]
                    for (int64_t i = 0; i < H.nf; ++i) fpf.push_back((int32_t)i);
                    for (int64_t i = 0; i < H.np; ++i) fpp.push_back((int32_t)(H.nf + i));
                }
                H.fs_fp = std::make_unique<PCFieldSplit>(H.Kfp, fpp, fpf, o, "fp_", c);
                H.ksp_fp = make_ksp("fp_", o, &H.Kfp, &H.Kfp, "gmres", "fieldsplit", c, 1e-5, 1e-50, 1e4, 10000, 30,
                                    H.fs_fp.get());
            } else {
                H.ksp_fp = make_ksp("fp_", o, &H.Kfp, &H.Kfp, "gmres", pt, c);
            }
        }
    }
fp_done:
    stage(H.three_way ? "f / p / diff block solvers" : "fp block solver");
    // the inner Anderson history lives as long as the preconditioner object
    // (lib/Preconditioner.py: created in __init__, not in setUp)
    if (!H.mixer_ready) {
        H.mixer.init((int)o.integer("pls.inner_accel_order", 0), n);
        H.mixer_ready = true;
    }
    H.bpc.h = &H;
    H.bpc.type = "python";
    H.bpc.n = n;
    alloc_work(H);
    if (!H.keep) {
        H.P = DevCSR();
        H.Pd = DevCSR();
    }
    c.sync();
    H.setup_done = true;
}


// lib/Solver.py:64-103 create_solver (after the PC exists, as in Poromechanics.py:62-67)
static void do_setup_solver(Handle &H) {
    if (H.solver_ready) return;
    Ctx &c = H.ctx;
    const Options &o = H.opt;
    const int64_t n = H.n;
    H.solver_type = o.str("pls.solver_type", "gmres");
    const double atol = o.num("pls.solver_atol", 1e-8), rtol = o.num("pls.solver_rtol", 1e-6);
    const int64_t maxiter = o.integer("pls.solver_maxiter", 500);
    H.A.tag = 1;
    build_sell(H.A, c);
    H.Aop = std::make_unique<MatOp>(&H.A);
    H.Aop->timers = &H.timers;
    if (H.solver_type == "aar") {
        auto &a = H.aar;
        a.order = (int)o.integer("pls.aar_order", 10);
        a.p = (int)o.integer("pls.aar_p", 5);
        a.omega = o.num("pls.aar_omega", 1.0);
        a.beta = o.num("pls.aar_beta", 1.0);
        a.atol = atol;
        a.rtol = rtol;
        a.maxiter = maxiter;
        a.monitor = o.flag("pls.solver_monitor", false);
        if (a.order > 15) throw Error("AAR order > 15 not supported");
        a.F.init(a.order + 1, n);
        a.X.init(a.order + 1, n);
        a.xk.alloc(n); a.fk.alloc(n); a.dxk.alloc(n); a.dfk.alloc(n); a.tmp.alloc(n);
        a.pX.alloc(16); a.pF.alloc(16); a.dalpha.alloc(16);
    } else {
        const int64_t restart = (H.solver_type == "gmres") ? maxiter : 30;
        H.outer = make_ksp("global_", o, &H.A, nullptr, H.solver_type, "python", c, rtol, atol, 1e20, maxiter, restart,
                           &H.bpc);
        H.outer->owned_op.reset();
        H.outer->A = H.Aop.get();
        H.outer->monitor = H.outer->monitor || o.flag("pls.solver_monitor", false);
        const std::string gpc = o.str("global_pc_type", "python");
        if (gpc != "python") throw Error("global_pc_type must stay 'python' (the block preconditioner)");
    }
    c.sync();
    H.solver_ready = true;
}

// ---------------------------------------------------------------- AAR -----
// lib/AAR.py:46-128 (single process: the rank-0 gathers are the identity).
static void aar_solve(Handle &H, const double *b, double *x) {
    Ctx &c = H.ctx;
    auto &a = H.aar;
    const int64_t n = H.n;
    // x0 = 0; fk = b - A x0 = b
    launch_set(n, 0.0, a.xk.p, c.st);
    launch_copy(n, b, a.fk.p, c.st);
    const double error0 = c.norm2(n, a.fk.p);
    double err_abs = error0, err_rel = 1.0;
    int64_t it = 0;
    H.history.assign(1, error0);
    while (err_abs > a.atol && err_rel > a.rtol && it < a.maxiter) {
        launch_copy(n, a.fk.p, a.dfk.p, c.st);
        launch_copy(n, a.xk.p, a.dxk.p, c.st);
        // update_residual: temp = b - A xk ; fk = PC(temp)
        H.Aop->apply(a.xk.p, a.tmp.p, c);
        launch_waxpby(n, 1.0, b, -1.0, a.tmp.p, a.tmp.p, c.st);
        H.bpc.apply(a.tmp.p, a.fk.p, c);
        launch_waxpby(n, 1.0, a.fk.p, -1.0, a.dfk.p, a.dfk.p, c.st);  // dfk = fk - dfk
        a.F.append(a.dfk.p, a.order, c);
        const double fnorm = c.norm2(n, a.fk.p);
        const char *kind = "R";
        if (fnorm < 1e-14) {
            // no update (AAR.py:91-92)
        } else if (it == 0 || a.order == 0 || ((it + 1) % a.p) != 0) {
            launch_axpby(n, a.omega, a.fk.p, 1.0, a.xk.p, c.st);
        } else {
            kind = "A";
            const int64_t mk = std::min<int64_t>(a.order, it);
            std::vector<const double *> cols;
            for (int i = 0; i < a.F.size(); ++i) cols.push_back(a.F.at(i));
            std::vector<double> alpha = a.ls.solve(cols, a.fk.p, n, c);
            if ((int64_t)a.X.size() < mk) throw Error("AAR: history shorter than mk");
            std::vector<const double *> hx, hf;
            for (int64_t i = 0; i < mk; ++i) { hx.push_back(a.X.at((int)i)); hf.push_back(a.F.at((int)i)); }
            if (mk > 0) {
                HIPCHK(hipMemcpyAsync((void *)a.pX.p, hx.data(), sizeof(double *) * mk, hipMemcpyHostToDevice, c.st));
                HIPCHK(hipMemcpyAsync((void *)a.pF.p, hf.data(), sizeof(double *) * mk, hipMemcpyHostToDevice, c.st));
                HIPCHK(hipMemcpyAsync(a.dalpha.p, alpha.data(), sizeof(double) * mk, hipMemcpyHostToDevice, c.st));
            }
            k_anderson_update<<<2048, 256, 0, c.st>>>(n, (int)mk, a.pX.p, a.pF.p, a.dalpha.p, a.beta, a.fk.p, a.xk.p);
            c.sync();
        }
        launch_waxpby(n, 1.0, a.xk.p, -1.0, a.dxk.p, a.dxk.p, c.st);  // dxk = xk - dxk
        a.X.append(a.dxk.p, a.order, c);
        err_abs = fnorm;
        err_rel = err_abs / error0;
        it += 1;
        H.history.push_back(err_abs);
        if (a.monitor) printf("---- Iteration [%s] %3lld\tabs=%1.2e\trel=%1.2e\n", kind, (long long)it, err_abs, err_rel);
        H.timers.flush();
    }
    launch_copy(n, a.xk.p, x, c.st);
    c.sync();
    H.res.its = (int)it;
    H.res.rnorm = err_abs;
    H.res.reason = (err_abs <= a.atol) ? 3 : (err_rel <= a.rtol) ? 2 : -3;
}

static void solve_device(Handle &H, const double *b, double *x) {
    do_setup(H);
    do_setup_solver(H);
    Ctx &c = H.ctx;
    H.pc_applies = 0;
    H.timers.begin(T_SOLVER);
    if (H.solver_type == "aar") {
        aar_solve(H, b, x);
    } else {
        H.outer->solve(b, x, c);
        H.res.its = H.outer->its;
        H.res.reason = H.outer->reason;
        H.res.rnorm = H.outer->rnorm;
        H.history = H.outer->history;
    }
    H.timers.end(T_SOLVER);
    c.sync();
    H.timers.flush();
    H.res.pc_applies = H.pc_applies;
    H.res.history_len = (int32_t)H.history.size();
}

}  // namespace pls

// ======================================================== extern "C" ABI ===
using namespace pls;

#define PLS_TRY(...)                                            \
    try {                                                       \
        __VA_ARGS__;                                            \
        return 0;                                               \
    } catch (const std::exception &e) {                         \
        g_last_error = e.what();                                \
        return 1;                                               \
    } catch (...) {                                             \
        g_last_error = "unknown error";                         \
        return 1;                                               \
    }

extern "C" {

int pls_abi_version(void) { return PLS_ABI_VERSION; }
const char *pls_last_error(void) { return g_last_error.c_str(); }

int pls_device_count(int *count) {
    PLS_TRY({
        int c = 0;
        hipError_t e = hipGetDeviceCount(&c);
        if (e != hipSuccess) c = 0;
        *count = c;
    })
}
int pls_set_device(int device) { PLS_TRY(HIPCHK(hipSetDevice(device))) }

static void check_is(const int32_t *is, int64_t m, int64_t n, std::vector<char> &seen, const char *name) {
    for (int64_t i = 0; i < m; ++i) {
        if (is[i] < 0 || is[i] >= n) throw Error(std::string(name) + ": index out of range");
        if (i && is[i] <= is[i - 1]) throw Error(std::string(name) + ": must be sorted ascending and unique");
        if (seen[is[i]]) throw Error(std::string(name) + ": overlaps another field");
        seen[is[i]] = 1;
    }
}

int pls_create(const pls_csr *A, const pls_csr *P, const pls_csr *Pdiff, const int32_t *is_s, int64_t ns,
               const int32_t *is_f, int64_t nf, const int32_t *is_p, int64_t np, const int32_t *bcs_sub_p, int64_t nbc,
               const char *options, pls_handle **out) {
    PLS_TRY({
        if (!A || !P || !out) throw Error("pls_create: A, P and out are required");
        {
            Options pre;
            pre.parse(options);
            validate_pc_type(pre);
        }
        auto H = std::make_unique<Handle>();
        H->opt.parse(options);
        H->parse_params();
        H->timers.st = H->ctx.st;
        H->ns = ns; H->nf = nf; H->np = np; H->n = ns + nf + np;
        const int64_t n = H->n;
        std::vector<char> seen(n, 0);
        check_is(is_s, ns, n, seen, "is_s");
        check_is(is_f, nf, n, seen, "is_f");
        check_is(is_p, np, n, seen, "is_p");
        // internal order: 2-way [is_s | is_fp = sorted(f U p)], 3-way [is_s | is_f | is_p]
        H->perm.assign(is_s, is_s + ns);
        if (H->three_way) {
            H->perm.insert(H->perm.end(), is_f, is_f + nf);
            H->perm.insert(H->perm.end(), is_p, is_p + np);
        } else {
            std::vector<int64_t> fp(is_f, is_f + nf);
            fp.insert(fp.end(), is_p, is_p + np);
            std::sort(fp.begin(), fp.end());
            H->perm.insert(H->perm.end(), fp.begin(), fp.end());
            std::vector<char> isf(n, 0);
            for (int64_t i = 0; i < nf; ++i) isf[is_f[i]] = 1;
            for (size_t t = 0; t < fp.size(); ++t) (isf[fp[t]] ? H->fp_is_f : H->fp_is_p).push_back((int32_t)t);
        }
        std::vector<int64_t> inv(n);
        for (int64_t i = 0; i < n; ++i) inv[H->perm[i]] = i;
        upload_permuted(A, *H, inv, H->A);
        upload_permuted(P, *H, inv, H->P);
        if (Pdiff) {
            upload_permuted(Pdiff, *H, inv, H->Pd);
            H->have_Pd = true;
        }
        H->dperm.alloc(std::max<int64_t>(n, 1));
        HIPCHK(hipMemcpy(H->dperm.p, H->perm.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice));
        H->bcs.assign(bcs_sub_p, bcs_sub_p + nbc);
        for (int32_t b : H->bcs)
            if (b < 0 || b >= np) throw Error("bcs_sub_pressure: position out of range of the p sub-vector");
        H->dbcs.alloc(std::max<int64_t>(nbc, 1));
        if (nbc) HIPCHK(hipMemcpy(H->dbcs.p, H->bcs.data(), sizeof(int32_t) * nbc, hipMemcpyHostToDevice));
        H->keep = H->opt.flag("pls.keep_matrices", true);
        *out = reinterpret_cast<pls_handle *>(H.release());
    })
}

// Synthetic system generated directly in HBM.  With a communicator of size G
// every rank generates only its row slabs (global columns), then the
// matrices become distributed (make_dist): the same global system, sharded.
static Handle *create_synthetic(const pls_synth_spec *spec, const char *options, Comm *comm) {
    {
        Options pre;
        pre.parse(options);
        validate_pc_type(pre);
    }
    auto H = std::make_unique<Handle>();
    H->opt.parse(options);
    H->parse_params();
    H->timers.st = H->ctx.st;
    if (comm) H->ctx.comm = comm;
    Comm *cm = H->ctx.comm;
    SynthHost S;
    S.init(*spec);
    H->dist.init(S.n, cm->rank, cm->size);
    H->distributed = cm->size > 1;
    const Dist &Dd = H->dist;
    H->ns = Dd.len[0]; H->nf = Dd.len[1]; H->np = Dd.len[2];
    H->n = Dd.nloc;
    const int64_t n = H->n;
    const int64_t nglob = S.n[0] + S.n[1] + S.n[2];
    Ctx &c = H->ctx;
    H->synth_offs.alloc(6 * 128);
    auto D = std::make_unique<SynthDev>();
    *D = SynthDev{};
    D->dim = S.dim;
    D->seed = S.seed;
    D->delta = S.delta;
    for (int f = 0; f < 3; ++f) {
        D->n[f] = S.n[f];
        D->off[f] = S.off[f];
        D->rlo[f] = Dd.lo[f];
        D->rlen[f] = Dd.len[f];
        D->rloff[f] = Dd.loff[f];
    }
    D->nrows = n;
    for (int b = 0; b < 6; ++b) {
        D->cnt[b] = S.cnt[b];
        HIPCHK(hipMemcpy(H->synth_offs.p + b * 128, S.offs[b].data(), sizeof(int32_t) * S.cnt[b],
                         hipMemcpyHostToDevice));
        D->offs[b] = H->synth_offs.p + b * 128;
    }
    // pattern (shared by A, P, P_diff)
    DBuf<int64_t> len(n + 1);
    launch_synth_count(*D, len.p, c.st);
    H->A.rp.alloc(n + 1);
    c.ensure_scan(n);
    exclusive_scan_i64(len.p, H->A.rp.p, n, c.scan_tmp.p, c.scan_tmp_bytes, c.st);
    int64_t nnz = 0;
    HIPCHK(hipMemcpyAsync(&nnz, H->A.rp.p + n, sizeof(int64_t), hipMemcpyDeviceToHost, c.st));
    c.sync();
    auto gen = [&](DevCSR &M, int variant) {
        M.nrows = n; M.ncols = nglob; M.nnz = nnz;
        if (!M.rp.p) {
            M.rp.alloc(n + 1);
            HIPCHK(hipMemcpyAsync(M.rp.p, H->A.rp.p, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToDevice, c.st));
        }
        M.ci.alloc(std::max<int64_t>(nnz, 1));
        M.val.alloc(std::max<int64_t>(nnz, 1));
        launch_synth_fill(*D, variant, M.rp.p, M.ci.p, M.val.p, c.st);
        HIPCHK(hipGetLastError());
    };
    gen(H->A, 0);
    gen(H->P, 1);
    if (H->three_way) {
        gen(H->Pd, 2);
        H->have_Pd = true;
    }
    c.sync();
    if (H->distributed) make_dist(H->A, Dd, 0, 2, cm, c);
    H->perm.resize(n);
    std::iota(H->perm.begin(), H->perm.end(), 0);
    H->dperm.alloc(std::max<int64_t>(n, 1));
    HIPCHK(hipMemcpy(H->dperm.p, H->perm.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice));
    for (int64_t i = Dd.lo[2]; i < Dd.lo[2] + Dd.len[2]; ++i)
        if (S.is_bc(i)) H->bcs.push_back((int32_t)(i - Dd.lo[2]));
    H->dbcs.alloc(std::max<size_t>(H->bcs.size(), 1));
    if (!H->bcs.empty())
        HIPCHK(hipMemcpy(H->dbcs.p, H->bcs.data(), sizeof(int32_t) * H->bcs.size(), hipMemcpyHostToDevice));
    H->keep = H->opt.flag("pls.keep_matrices", nnz < 50000000);
    H->synth_rows = std::move(D);
    return H.release();
}

int pls_create_synthetic(const pls_synth_spec *spec, const char *options, pls_handle **out) {
    PLS_TRY(*out = reinterpret_cast<pls_handle *>(create_synthetic(spec, options, nullptr)))
}

int pls_create_synthetic_dist(const pls_synth_spec *spec, const char *options, pls_comm *comm, pls_handle **out) {
    PLS_TRY({
        if (!comm) throw Error("pls_create_synthetic_dist: communicator required");
        *out = reinterpret_cast<pls_handle *>(create_synthetic(spec, options, reinterpret_cast<Comm *>(comm)));
    })
}

// Multi-rank drop-in from caller matrices: the reference runs under
// `mpirun -np 8` (paper-scripts/robustness_2d.sh:29) where every rank holds the
// MPIAIJ rows it owns (A.getValuesCSR() of lib/Solver.py:151's operator: local
// rows, global columns) and the index sets of the dofs it owns
// (lib/IndexSet.py:38-49).  PETSc's createSubMatrix (lib/Preconditioner.py:
// 61-74) then gives every field block the row ownership of the rank-local IS
// entries; the same here: field f of rank q is the contiguous internal range
// start[f][q] .. start[f][q+1] (3-way fields s, f, p; 2-way s and
// fp = sorted(f U p), PETSc's is_fp), columns renumbered to that field-major
// global order, then make_dist builds the halo plan as for synthetic shards.
static Handle *create_dist(const pls_csr *A, const pls_csr *P, const pls_csr *Pdiff, int64_t row_start,
                           const int32_t *is_s, int64_t ns, const int32_t *is_f, int64_t nf, const int32_t *is_p,
                           int64_t np, const int32_t *bcs_sub_p, int64_t nbc, const char *options, Comm *cm) {
    if (!A || !P) throw Error("pls_create_dist: A and P are required");
    {
        Options pre;
        pre.parse(options);
        validate_pc_type(pre);
    }
    auto H = std::make_unique<Handle>();
    H->opt.parse(options);
    H->parse_params();
    H->timers.st = H->ctx.st;
    H->ctx.comm = cm;
    Ctx &c = H->ctx;
    const int G = cm->size, r = cm->rank;
    const int64_t nloc = ns + nf + np;
    if (A->nrows != nloc || P->nrows != nloc || (Pdiff && Pdiff->nrows != nloc))
        throw Error("pls_create_dist: local matrices must have ns + nf + np rows (this rank's rows)");
    // this rank's rows are [row_start, row_start + nloc) of the caller's numbering
    std::vector<char> seen(nloc, 0);
    auto check_local = [&](const int32_t *is, int64_t m, const char *name) {
        for (int64_t i = 0; i < m; ++i) {
            const int64_t l = (int64_t)is[i] - row_start;
            if (l < 0 || l >= nloc) throw Error(std::string(name) + ": index not owned by this rank");
            if (i && is[i] <= is[i - 1]) throw Error(std::string(name) + ": must be sorted ascending and unique");
            if (seen[l]) throw Error(std::string(name) + ": overlaps another field");
            seen[l] = 1;
        }
    };
    check_local(is_s, ns, "is_s");
    check_local(is_f, nf, "is_f");
    check_local(is_p, np, "is_p");
    // internal local order and the field counts the Dist sees
    std::vector<int64_t> order(is_s, is_s + ns);  // caller global indices in internal local order
    int64_t cnt[3] = {ns, nf, np};
    if (H->three_way) {
        order.insert(order.end(), is_f, is_f + nf);
        order.insert(order.end(), is_p, is_p + np);
    } else {
        std::vector<int64_t> fp(is_f, is_f + nf);
        fp.insert(fp.end(), is_p, is_p + np);
        std::sort(fp.begin(), fp.end());
        std::vector<char> isf(nloc, 0);
        for (int64_t i = 0; i < nf; ++i) isf[is_f[i] - row_start] = 1;
        for (size_t t = 0; t < fp.size(); ++t) (isf[fp[t] - row_start] ? H->fp_is_f : H->fp_is_p).push_back((int32_t)t);
        order.insert(order.end(), fp.begin(), fp.end());
        cnt[1] = nf + np;
        cnt[2] = 0;
    }
    // every rank's field counts -> ownership ranges of the internal numbering
    std::vector<int64_t> all((size_t)3 * G);
    cm->allgather_host(cnt, sizeof(int64_t) * 3, all.data());
    std::vector<int64_t> counts[3];
    int64_t maxloc = 0;
    for (int f = 0; f < 3; ++f) counts[f].resize(G);
    for (int q = 0; q < G; ++q) {
        int64_t t = 0;
        for (int f = 0; f < 3; ++f) t += (counts[f][q] = all[(size_t)q * 3 + f]);
        maxloc = std::max(maxloc, t);
    }
    H->dist.init_counts(counts, r, G);
    const Dist &D = H->dist;
    const int64_t nglob = D.n[0] + D.n[1] + D.n[2];
    if (A->ncols != nglob || P->ncols != nglob || (Pdiff && Pdiff->ncols != nglob))
        throw Error("pls_create_dist: matrix columns must span the global system (sum of every rank's rows)");
    // caller global index -> internal global index, from every rank's order
    std::vector<int64_t> mine(maxloc, -1), every((size_t)maxloc * G);
    std::copy(order.begin(), order.end(), mine.begin());
    cm->allgather_host(mine.data(), sizeof(int64_t) * maxloc, every.data());
    std::vector<int32_t> cmap(nglob, -1);
    for (int q = 0; q < G; ++q) {
        int64_t k = 0;
        for (int f = 0; f < 3; ++f)
            for (int64_t i = 0; i < counts[f][q]; ++i, ++k) {
                const int64_t g = every[(size_t)q * maxloc + k];
                if (g < 0 || g >= nglob || cmap[g] >= 0) throw Error("pls_create_dist: index sets do not partition 0..n-1");
                cmap[g] = (int32_t)(D.off[f] + D.start[f][q] + i);
            }
    }
    // local rows in internal order, columns in the internal global numbering
    auto upload = [&](const pls_csr *M, DevCSR &out) {
        std::vector<int64_t> rp(nloc + 1, 0);
        for (int64_t i = 0; i < nloc; ++i) {
            const int64_t o = order[i] - row_start;
            rp[i + 1] = rp[i] + (M->row_ptr[o + 1] - M->row_ptr[o]);
        }
        std::vector<int32_t> ci(rp[nloc]);
        std::vector<double> v(rp[nloc]);
        std::vector<std::pair<int32_t, double>> row;
        for (int64_t i = 0; i < nloc; ++i) {
            const int64_t o = order[i] - row_start;
            row.clear();
            for (int64_t k = M->row_ptr[o]; k < M->row_ptr[o + 1]; ++k) {
                const int32_t cc = M->col[k];
                if (cc < 0 || cc >= nglob) throw Error("pls_create_dist: column index out of range");
                row.emplace_back(cmap[cc], M->val[k]);
            }
            std::sort(row.begin(), row.end(), [](auto &a, auto &b) { return a.first < b.first; });
            for (size_t t = 0; t < row.size(); ++t) {
                ci[rp[i] + t] = row[t].first;
                v[rp[i] + t] = row[t].second;
            }
        }
        upload_csr(out, nloc, nglob, rp.data(), ci.data(), v.data(), c);
    };
    upload(A, H->A);
    upload(P, H->P);
    if (Pdiff) {
        upload(Pdiff, H->Pd);
        H->have_Pd = true;
    }
    H->ns = ns; H->nf = nf; H->np = np; H->n = nloc;
    H->distributed = G > 1;
    if (H->distributed) make_dist(H->A, D, 0, 2, cm, c);
    H->perm.resize(nloc);
    for (int64_t i = 0; i < nloc; ++i) H->perm[i] = order[i] - row_start;
    H->dperm.alloc(std::max<int64_t>(nloc, 1));
    HIPCHK(hipMemcpy(H->dperm.p, H->perm.data(), sizeof(int64_t) * nloc, hipMemcpyHostToDevice));
    // bcs_sub_pressure: positions inside this rank's p sub-vector (what
    // Poromechanics.py:48-55 computes from the rank's own dofs)
    H->bcs.assign(bcs_sub_p, bcs_sub_p + nbc);
    for (int32_t b : H->bcs)
        if (b < 0 || b >= np) throw Error("bcs_sub_pressure: position out of range of the p sub-vector");
    H->dbcs.alloc(std::max<int64_t>(nbc, 1));
    if (nbc) HIPCHK(hipMemcpy(H->dbcs.p, H->bcs.data(), sizeof(int32_t) * nbc, hipMemcpyHostToDevice));
    H->keep = H->opt.flag("pls.keep_matrices", true);
    return H.release();
}

int pls_create_dist(const pls_csr *A, const pls_csr *P, const pls_csr *Pdiff, int64_t row_start, const int32_t *is_s,
                    int64_t ns, const int32_t *is_f, int64_t nf, const int32_t *is_p, int64_t np,
                    const int32_t *bcs_sub_p, int64_t nbc, const char *options, pls_comm *comm, pls_handle **out) {
    PLS_TRY({
        if (!comm || !out) throw Error("pls_create_dist: communicator and out are required");
        *out = reinterpret_cast<pls_handle *>(create_dist(A, P, Pdiff, row_start, is_s, ns, is_f, nf, is_p, np,
                                                          bcs_sub_p, nbc, options, reinterpret_cast<Comm *>(comm)));
    })
}

int pls_rccl_unique_id(char out[128]) { PLS_TRY(rccl_unique_id(out)) }
int pls_comm_create_rccl(const char id[128], int rank, int size, pls_comm **out) {
    PLS_TRY(*out = reinterpret_cast<pls_comm *>(static_cast<Comm *>(rccl_init(id, rank, size))))
}
int pls_comm_create_callback(int rank, int size, pls_allgather_fn fn, void *user, pls_comm **out) {
    PLS_TRY({
        if (!fn || rank < 0 || rank >= size) throw Error("pls_comm_create_callback: bad arguments");
        auto *cb = new CommCallback();
        cb->rank = rank;
        cb->size = size;
        cb->fn = fn;
        cb->user = user;
        *out = reinterpret_cast<pls_comm *>(static_cast<Comm *>(cb));
    })
}
int pls_comm_destroy(pls_comm *comm) { PLS_TRY(delete reinterpret_cast<Comm *>(comm)) }

int pls_setup(pls_handle *h) { PLS_TRY(do_setup(*reinterpret_cast<Handle *>(h))) }
int pls_destroy(pls_handle *h) { PLS_TRY(delete reinterpret_cast<Handle *>(h)) }
int pls_set_option(pls_handle *hh, const char *key, const char *value) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        std::string k(key ? key : "");
        while (!k.empty() && k[0] == '-') k.erase(0, 1);
        if (k.empty()) throw Error("pls_set_option: empty key");
        const bool solver_key = k.rfind("pls.solver", 0) == 0 || k.rfind("pls.aar", 0) == 0 || k.rfind("global_", 0) == 0;
        if (solver_key && H.solver_ready) throw Error("option " + k + " set after the solver was created");
        if (!solver_key && H.setup_done) throw Error("option " + k + " set after the preconditioner was set up");
        H.opt.kv[k] = value ? value : "";
        if (k == "pls.timers") H.timers.enabled = H.opt.flag(k, true);
    })
}
int pls_create_solver(pls_handle *hh) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        do_setup(H);
        do_setup_solver(H);
    })
}

int pls_get_sizes(pls_handle *hh, int64_t *n, int64_t *ns, int64_t *nf, int64_t *np, int64_t *nnz_A) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        if (n) *n = H.n;
        if (ns) *ns = H.ns;
        if (nf) *nf = H.nf;
        if (np) *np = H.np;
        if (nnz_A) *nnz_A = H.A.nnz;
    })
}

static void to_internal(Handle &H, const double *x_host, double *d_internal) {
    HIPCHK(hipMemcpyAsync(H.vout.p, x_host, sizeof(double) * H.n, hipMemcpyHostToDevice, H.ctx.st));
    launch_gather(H.n, H.dperm.p, H.vout.p, d_internal, H.ctx.st);
}
static void from_internal(Handle &H, const double *d_internal, double *y_host) {
    launch_scatter(H.n, H.dperm.p, d_internal, H.vout.p, H.ctx.st);
    HIPCHK(hipMemcpyAsync(y_host, H.vout.p, sizeof(double) * H.n, hipMemcpyDeviceToHost, H.ctx.st));
    H.ctx.sync();
}

int pls_pc_apply(pls_handle *hh, const double *x, double *y) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        do_setup(H);
        DBuf<double> xi(H.n), yi(H.n);
        to_internal(H, x, xi.p);
        H.bpc.apply(xi.p, yi.p, H.ctx);
        from_internal(H, yi.p, y);
        H.timers.flush();
    })
}

int pls_matmult(pls_handle *hh, const double *x, double *y) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        DBuf<double> xi(H.n), yi(H.n);
        if (!H.vout.p) H.vout.alloc(H.n);
        to_internal(H, x, xi.p);
        build_sell(H.A, H.ctx);
        spmv(H.A, xi.p, yi.p, H.ctx);
        from_internal(H, yi.p, y);
    })
}

int pls_solve(pls_handle *hh, const double *b, double *x, pls_result *res) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        do_setup(H);
        DBuf<double> bi(H.n), xi(H.n);
        to_internal(H, b, bi.p);
        solve_device(H, bi.p, xi.p);
        from_internal(H, xi.p, x);
        if (res) *res = H.res;
    })
}

int pls_solve_device(pls_handle *hh, const double *d_b, double *d_x, pls_result *res) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        solve_device(H, d_b, d_x);
        if (res) *res = H.res;
    })
}
int pls_pc_apply_device(pls_handle *hh, const double *d_x, double *d_y) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        do_setup(H);
        H.bpc.apply(d_x, d_y, H.ctx);
        H.ctx.sync();
        H.timers.flush();
    })
}
int pls_matmult_device(pls_handle *hh, const double *d_x, double *d_y) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        build_sell(H.A, H.ctx);
        spmv(H.A, d_x, d_y, H.ctx);
        H.ctx.sync();
    })
}
int pls_synthetic_rhs_device(pls_handle *hh, uint64_t seed, double *d_b) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        if (!H.synth_rows) throw Error("pls_synthetic_rhs_device: not a synthetic handle");
        launch_synth_rhs(*H.synth_rows, seed, d_b, H.ctx.st);
        H.ctx.sync();
    })
}
int pls_device_alloc(int64_t bytes, void **d_ptr) { PLS_TRY(HIPCHK(hipMalloc(d_ptr, (size_t)bytes))) }
int pls_device_free(void *d_ptr) { PLS_TRY(HIPCHK(hipFree(d_ptr))) }
int pls_memcpy_h2d(void *d_dst, const void *h_src, int64_t bytes) {
    PLS_TRY(HIPCHK(hipMemcpy(d_dst, h_src, (size_t)bytes, hipMemcpyHostToDevice)))
}
int pls_memcpy_d2h(void *h_dst, const void *d_src, int64_t bytes) {
    PLS_TRY(HIPCHK(hipMemcpy(h_dst, d_src, (size_t)bytes, hipMemcpyDeviceToHost)))
}

int pls_get_result(pls_handle *hh, pls_result *res) {
    PLS_TRY({ *res = reinterpret_cast<Handle *>(hh)->res; })
}
int pls_get_history(pls_handle *hh, double *hist, int32_t cap) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        const int32_t m = std::min<int32_t>(cap, (int32_t)H.history.size());
        std::copy(H.history.begin(), H.history.begin() + m, hist);
    })
}
int pls_get_timings(pls_handle *hh, pls_timings *t) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        H.timers.flush();
        t->pc_total = H.timers.acc[T_PC_TOTAL];
        t->pc_solid = H.timers.acc[T_PC_SOLID];
        t->pc_fluid = H.timers.acc[T_PC_FLUID];
        t->pc_press = H.three_way ? H.timers.acc[T_PC_PRESS] : H.timers.acc[T_PC_FLUID];
        t->pc_alloc = H.timers.acc[T_PC_ALLOC];
        t->solver_total = H.timers.acc[T_SOLVER];
        t->spmv_total = H.timers.acc[T_SPMV];
        t->spmv_calls = H.timers.spmv_calls;
    })
}
int pls_get_ksp_stats(pls_handle *hh, const char *prefix, int64_t *stats) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        if (!prefix || !stats) throw Error("pls_get_ksp_stats: null argument");
        const std::string want(prefix);
        const KSP *found = nullptr;
        std::vector<const KSP *> all = {H.ksp_s.get(), H.ksp_f.get(), H.ksp_p.get(), H.ksp_pd.get(), H.ksp_fp.get(),
                                        H.outer.get()};
        if (H.ksp_fp && H.ksp_fp->pc)
            if (const PCFieldSplit *fs = dynamic_cast<const PCFieldSplit *>(H.ksp_fp->pc)) {
                all.push_back(fs->k0.get());
                all.push_back(fs->k1.get());
            }
        if (H.fs_fp) {
            all.push_back(H.fs_fp->k0.get());
            all.push_back(H.fs_fp->k1.get());
        }
        for (const KSP *k : all)
            if (k && k->prefix == want) found = k;
        if (!found) throw Error("pls_get_ksp_stats: no inner solver with prefix '" + want + "'");
        stats[0] = found->stat_solves;
        stats[1] = found->stat_its;
        stats[2] = found->stat_max;
        stats[3] = found->stat_div;
        stats[4] = found->stat_last_neg;
    })
}
int pls_reset_timings(pls_handle *hh) { PLS_TRY(reinterpret_cast<Handle *>(hh)->timers.reset()) }

int pls_export_matrix(pls_handle *hh, int which, int64_t *nrows, int64_t *nnz, int64_t *row_ptr, int32_t *col,
                      double *val) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        const DevCSR &M = which == 0 ? H.A : which == 1 ? H.P : H.Pd;
        if (!M.rp.p) throw Error("matrix not available (freed after setup, or not generated)");
        *nrows = M.nrows;
        *nnz = M.nnz;
        if (col) {
            HIPCHK(hipMemcpy(row_ptr, M.rp.p, sizeof(int64_t) * (M.nrows + 1), hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(col, M.ci.p, sizeof(int32_t) * M.nnz, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(val, M.val.p, sizeof(double) * M.nnz, hipMemcpyDeviceToHost));
        }
    })
}
int pls_get_permutation(pls_handle *hh, int64_t *perm) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        std::copy(H.perm.begin(), H.perm.end(), perm);
    })
}

int pls_bench_spmv(pls_handle *hh, const double *d_x, double *d_y, int32_t reps, double *sec_per_launch) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        H.A.tag = 1;
        build_sell(H.A, H.ctx);
        hipEvent_t a, b;
        HIPCHK(hipEventCreate(&a));
        HIPCHK(hipEventCreate(&b));
        HIPCHK(hipEventRecord(a, H.ctx.st));
        for (int r = 0; r < reps; ++r) spmv(H.A, d_x, d_y, H.ctx);
        HIPCHK(hipEventRecord(b, H.ctx.st));
        HIPCHK(hipEventSynchronize(b));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, a, b));
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
        *sec_per_launch = (double)ms * 1e-3 / std::max(1, reps);
    })
}

// Host-only query of the classical-AMG setup (no device): level `level` of
// the hierarchy built from A with the options' prefix_pc_hypre_boomeramg_*
// values.  Outputs n, nc, P's nnz (the coarsest operator when level ==
// nlevels - 1); cf (n int8: 1 C, -1 F) and P's CSR arrays are written when
// non-NULL (call once for the sizes, then with buffers).
int pls_boomeramg_host_level(const pls_csr *A, const char *options, const char *prefix, int64_t level,
                             int64_t *nlevels, int64_t *n, int64_t *nc, int64_t *p_nnz, int8_t *cf, int64_t *p_rp,
                             int32_t *p_ci, double *p_v) {
    PLS_TRY({
        if (!A || A->nrows != A->ncols) throw Error("pls_boomeramg_host_level: square A required");
        Options o;
        o.parse(options);
        HostCSR H;
        H.nrows = H.ncols = A->nrows;
        H.rp.assign(A->row_ptr, A->row_ptr + A->nrows + 1);
        H.ci.assign(A->col, A->col + H.rp.back());
        H.v.assign(A->val, A->val + H.rp.back());
        std::vector<int8_t> cfv;
        HostCSR P;
        boomeramg_host_level(H, o, prefix ? prefix : "", level, *nlevels, *n, *nc, cfv, P);
        *p_nnz = (int64_t)P.ci.size();
        if (cf && !cfv.empty()) std::copy(cfv.begin(), cfv.end(), cf);
        if (p_rp && P.nrows > 0) std::copy(P.rp.begin(), P.rp.end(), p_rp);
        if (p_ci) std::copy(P.ci.begin(), P.ci.end(), p_ci);
        if (p_v) std::copy(P.v.begin(), P.v.end(), p_v);
    })
}

int pls_sparse_lu_analyze(const pls_csr *A, const char *options, double *stats, int64_t nstats, int32_t *perm,
                          int32_t *front_of, int32_t *parent) {
    PLS_TRY({
        if (!A || A->nrows != A->ncols) throw Error("pls_sparse_lu_analyze: square A required");
        if (A->nrows < 0 || !A->row_ptr || (A->nrows > 0 && !A->col))
            throw Error("pls_sparse_lu_analyze: negative size or null arrays");
        // the pattern is indexed directly by the symbolic analysis: validate it first
        if (A->row_ptr[0] != 0) throw Error("pls_sparse_lu_analyze: row_ptr[0] must be 0");
        for (int64_t i = 0; i < A->nrows; ++i)
            if (A->row_ptr[i + 1] < A->row_ptr[i]) throw Error("pls_sparse_lu_analyze: row_ptr must be nondecreasing");
        for (int64_t k = 0; k < A->row_ptr[A->nrows]; ++k)
            if (A->col[k] < 0 || A->col[k] >= A->ncols) throw Error("pls_sparse_lu_analyze: column index out of range");
        Options o;
        o.parse(options);
        HostCSR H;
        H.nrows = H.ncols = A->nrows;
        H.rp.assign(A->row_ptr, A->row_ptr + A->nrows + 1);
        H.ci.assign(A->col, A->col + H.rp.back());
        if (A->val) H.v.assign(A->val, A->val + H.rp.back());
        sparse_lu_analyze(H, o, stats, nstats, perm, front_of, parent);
    })
}

// Standalone AndersonAcceleration (lib/AndersonAcceleration.py:8-78) on its
// own stream and a single-rank communicator; the same mixer the block PC runs
// for "inner accel order" > 0.
struct AndersonObj {
    Ctx ctx;
    AndersonMixer mix;
};
int pls_anderson_create(int32_t order, int64_t n, pls_anderson **out) {
    PLS_TRY({
        if (!out) throw Error("pls_anderson_create: out is NULL");
        if (order < 0 || order > 15) throw Error("pls_anderson_create: order must be in 0..15");
        if (n < 0) throw Error("pls_anderson_create: negative length");
        auto *a = new AndersonObj();
        a->mix.init(order, n);
        *out = reinterpret_cast<pls_anderson *>(a);
    })
}
int pls_anderson_next(pls_anderson *aa, double *d_gk) {
    PLS_TRY({
        if (!aa) throw Error("pls_anderson_next: NULL object");
        AndersonObj &a = *reinterpret_cast<AndersonObj *>(aa);
        if (a.mix.n > 0 && !d_gk) throw Error("pls_anderson_next: NULL vector");
        // order 0: mk = 0 every call, x_k = g_k (AndersonAcceleration.py:69-70)
        if (a.mix.order > 0) a.mix.next(d_gk, a.ctx);
        a.ctx.sync();
    })
}
int pls_anderson_destroy(pls_anderson *a) { PLS_TRY(delete reinterpret_cast<AndersonObj *>(a)) }

// Latency of the solve's global sums (one batched all-reduce per
// CGS step, one per norm): reps x (global_sum_dev of `count` doubles + the
// stream sync the Krylov loop does to read them on the host), host clock.
int pls_bench_global_sum(pls_handle *hh, int32_t count, int32_t reps, double *sec_per_call) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        Ctx &c = H.ctx;
        if (count < 1 || count > 4096) throw Error("pls_bench_global_sum: count must be in 1..4096");
        DBuf<double> v(count);
        HIPCHK(hipMemsetAsync(v.p, 0, sizeof(double) * count, c.st));
        c.comm->global_sum_dev(v.p, count, c.st);  // warm (scratch allocation, first collective)
        c.sync();
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r) {
            c.comm->global_sum_dev(v.p, count, c.st);
            c.sync();
        }
        const auto t1 = std::chrono::steady_clock::now();
        *sec_per_call = std::chrono::duration<double>(t1 - t0).count() / std::max(1, reps);
    })
}

// New values (or patterns) of A, P, P_diff for the next solves, in the
// caller's ordering as for pls_create.  The block preconditioner is set up
// again before the next solve (PETSc re-runs PCSetUp when the operator state
// changes, as after the reference's bc.apply in every time step,
// lib/Poromechanics.py:70-86); the outer solver and AAR / inner Anderson
// histories persist, as the reference's objects do.
int pls_update_matrices(pls_handle *hh, const pls_csr *A, const pls_csr *P, const pls_csr *Pdiff) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        if (H.synth_rows) throw Error("pls_update_matrices: synthetic handles generate their matrices");
        if (H.distributed) throw Error("pls_update_matrices: not available for distributed handles");
        if (!P && !H.keep && H.setup_done)
            throw Error("pls_update_matrices: P was released after setup (pls.keep_matrices 0); pass P");
        const int64_t n = H.n;
        std::vector<int64_t> inv(n);
        for (int64_t i = 0; i < n; ++i) inv[H.perm[i]] = i;
        if (A) {
            upload_permuted(A, H, inv, H.A);
            H.A.sell.reset();
            H.A.tag = 1;
            if (H.solver_ready) build_sell(H.A, H.ctx);
        }
        if (P) upload_permuted(P, H, inv, H.P);
        if (Pdiff) {
            upload_permuted(Pdiff, H, inv, H.Pd);
            H.have_Pd = true;
        }
        H.setup_done = false;
    })
}

int pls_bench_copy(int64_t bytes, int32_t reps, int32_t read_only, double *gbs) {
    PLS_TRY({
        const int64_t n = std::max<int64_t>(bytes / 8, 2) & ~(int64_t)1;
        DBuf<double> a(n), b(n);
        hipStream_t st;
        HIPCHK(hipStreamCreate(&st));
        HIPCHK(hipMemsetAsync(a.p, 0, sizeof(double) * n, st));
        launch_copy_probe(n, a.p, b.p, read_only ? 1 : 0, st);
        hipEvent_t e0, e1;
        HIPCHK(hipEventCreate(&e0));
        HIPCHK(hipEventCreate(&e1));
        HIPCHK(hipEventRecord(e0, st));
        for (int r = 0; r < std::max(1, reps); ++r) launch_copy_probe(n, a.p, b.p, read_only ? 1 : 0, st);
        HIPCHK(hipEventRecord(e1, st));
        HIPCHK(hipEventSynchronize(e1));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, e0, e1));
        *gbs = (read_only ? 1.0 : 2.0) * 8.0 * (double)n * std::max(1, reps) / (ms * 1e-3) / 1e9;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipStreamDestroy(st);
    })
}

int pls_spmv_layout(pls_handle *hh, int32_t *d16, int64_t *matrix_bytes) {
    PLS_TRY({
        Handle &H = *reinterpret_cast<Handle *>(hh);
        build_sell(H.A, H.ctx);
        if (d16) *d16 = H.A.sell && H.A.sell->d16 ? 1 : 0;
        if (matrix_bytes) *matrix_bytes = H.A.sell ? H.A.sell->bytes() : 0;
    })
}

}  // extern "C"
