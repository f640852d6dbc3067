// runtime.hpp -- host runtime of libpls.so: device memory, options database,
// operators, preconditioners, Krylov solvers, the block preconditioner and
// AAR.  The Krylov loops run on the host over device-resident vectors; every
// vector operation is a HIP kernel on one stream, and the only device->host
// traffic per outer iteration is the handful of scalars the PETSc algorithms
// branch on (Hessenberg column, norms).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "comm.hpp"
#include "kernels.hpp"

namespace pls {

struct Error : std::runtime_error {
    explicit Error(const std::string &m) : std::runtime_error(m) {}
};

#define HIPCHK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess)                                                                       \
            throw ::pls::Error(std::string(#x) + " failed: " + hipGetErrorString(e_) + " at " +    \
                               __FILE__ + ":" + std::to_string(__LINE__));                          \
    } while (0)

// ------------------------------------------------------------ device buffer --
template <class T>
struct DBuf {
    T *p = nullptr;
    size_t n = 0;
    DBuf() = default;
    explicit DBuf(size_t count) { alloc(count); }
    DBuf(const DBuf &) = delete;
    DBuf &operator=(const DBuf &) = delete;
    DBuf(DBuf &&o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    DBuf &operator=(DBuf &&o) noexcept {
        if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
        return *this;
    }
    ~DBuf() { release(); }
    void alloc(size_t count) {
        release();
        n = count;
        if (count) HIPCHK(hipMalloc((void **)&p, sizeof(T) * count));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    T *get() const { return p; }
};

// ------------------------------------------------------------------ context --
struct Ctx {
    hipStream_t st = nullptr;
    Comm *comm = nullptr;   // global reductions (CommSelf unless distributed)
    DBuf<double> partial;   // reduction partials (NB_MAX (4096) x 136 at first; ensure_partial grows it)
    int64_t partial_n = 0;
    int64_t hscal_n = 0;    // doubles in the pinned host mirror
    DBuf<double> dscal;     // device scalars
    double *hscal = nullptr;  // pinned host mirror
    bool sell_d16 = true;     // build SpMV layouts as SELL-64/D16 where every row fits
    int d16_wide_lpr = 8;     // lanes per row of D16 slices with wide rows (option pls.d16_wide_lpr)
    int d16_unroll = 4;       // D16 SpMV 8-entry groups per lane in flight (option pls.d16_unroll)
    int d16_segs = D16_SEG;   // minimum D16 segment bases per lane (option pls.d16_segs; 8 where needed)
    int d16_sigma = 1024;         // SELL-C-sigma window (rows sorted by length; 0: never) (pls.d16_sigma)
    double d16_sigma_pad = 0.15;  // ... used when the plain plan pads more than this fraction (pls.d16_sigma_pad)
    int d16_sorted_lpr = 2;       // lanes per row of sorted slices with 32+ entries per row (pls.d16_sorted_lpr)
    bool spmv_b3 = false;         // row-triple layout for FE vector fields (pls.spmv_b3; measured slower)
    int spmv_rcm = -1;            // RCM-relabelled SpMV layout: -1 where the plain plan pads (FE), 0 never, 1 always
    int sweep_chain = -1;         // LDS-resident ILU / Gauss-Seidel blocks swept by one wave (k_ilu_blocks_chain):
                                  // -1 where the level DAG is deep and narrow, 0 never, 1 whenever rows fit
    int sweep_window = -1;        // ... in 64-row windows with inverted window triangles (k_ilu_blocks_window):
                                  // -1 where the chain sweep would be chosen, 0 never, 1 whenever rows fit
    int ilu_factor_dep = 1;       // ILU(0) factorization in one dependency-driven launch: 1 narrow levels, 2 always, 0 never
    int ilu_view = 0;             // print every ILU / Gauss-Seidel PC's sweep choice to stderr (pls.ilu_view)
    int ilu0_stage_cap = -1;      // test knob (pls.ilu0_stage): staged entries of the ILU(0) factorization, -1 default
    int ilu_dep_grid = 0;         // test knob (pls.ilu_dep_grid): k_ilu0_dep's persistent grid capped (0: none)
    int window_depth = 2;         // window sweep: windows of data in flight, 2 or 3 (pls.window_depth)
    int window_ring = -1;         // ... its ring variant for blocks longer than LDS (pls.window_ring: -1 where the
                                  // window sweep's level test holds, 0 off, 1 also forced on LDS-resident blocks)
    int window_kpw = 0;           // window sweep: stream records per wave (pls.window_kpw: 0 by the rows, 8 forced)
    int window_mixed = -1;        // ... its L triangle by levels (pls.window_mixed: -1 where L has no more levels
                                  // than windows, 0 off, 1 forced)
    int sweep_swin = 0;           // blocks too long for LDS: the super-window sweep (k_ilu_blocks_swin, experimental,
                                  // measured slower than the ring sweep): 0 never (default, capi), -1 where the ring
                                  // sweep would run, 1 whenever the block is y-resident
    double amg_csr_below = 16.0;  // AMG operators with fewer entries per row than this stay CSR (pls.amg_csr_below)
    bool halo_overlap = true;     // distributed SpMV: interior slices overlap the halo exchange (pls.halo_overlap)
    hipStream_t st_comm = nullptr;  // stream of the overlapped halo exchange (created on first use)
    hipEvent_t ev_x = nullptr, ev_halo = nullptr;
    DBuf<char> scan_tmp;
    size_t scan_tmp_bytes = 0;
    DBuf<double> rcm_x;  // x in RCM order for RCM-relabelled SpMV layouts (grown at layout build)
    // a redundant PC's gathered block: the rows each rank owns (contiguous, rank
    // order; empty when not) -- the classical AMG builds hypre's np = G hierarchy
    std::vector<int64_t> rank_rows;
    Ctx();
    ~Ctx();
    void sync() { HIPCHK(hipStreamSynchronize(st)); }
    void ensure_scan(int64_t n);
    // room for `cols` reductions of n entries (CGS: one partial per column and block) and
    // for `cols` + 2 doubles in the host mirror; setup only (frees the old buffers)
    void ensure_partial(int64_t n, int64_t cols);
    // every launch that writes `partial` / `hscal` takes its pointer from these:
    // they throw Error when the request exceeds the room (the round-3 fault was a
    // silent overrun of `partial` by a 453-column CGS block)
    double *partials(int64_t n, int64_t cols);
    double *host_scalars(int64_t count);
    // pls.debug_bounds: a canary region behind `partial` (checked by check_bounds,
    // which throws Error when it was written); pls.debug_partial_cap /
    // pls.debug_no_grow / pls.debug_unguarded reproduce the round-3 overrun in tests
    bool debug_bounds = false, debug_no_grow = false, debug_unguarded = false;
    static constexpr int64_t CANARY = 1 << 16;
    void set_debug(bool bounds, int64_t cap, bool no_grow, bool unguarded);
    void check_bounds();
    // deterministic reductions returning host values (synchronising)
    double dot(int64_t n, const double *x, const double *y);
    double norm2(int64_t n, const double *x);
};

// ------------------------------------------------------------------ matrix --
struct DevSELL {
    int64_t nslices = 0, stored = 0;  // stored = padded entries
    bool d16 = false;                 // SELL-64/D16: 16-bit column deltas (dl, seg) instead of col
    DBuf<int64_t> sptr;
    DBuf<int32_t> col;
    DBuf<double> val;
    DBuf<uint16_t> dl;
    DBuf<int32_t> seg, slpr;  // D16: segment bases per lane, lanes per row per slice
    DBuf<int64_t> sfirst;     // D16: first row of each slice (nslices + 1)
    int64_t wide_slices = 0;  // D16 slices with 8 lanes per row
    // SELL-C-sigma: slice positions hold rows sorted by length inside windows of
    // sigma rows (rowmap[position] = row); empty when rows keep their order
    DBuf<int32_t> rowmap;
    int64_t nrows_mapped = 0;
    // SELL/B3 (FE vector fields): row triples with one shared column list, lane =
    // triple; the D16 part above then holds only the other rows (through rowmap)
    int64_t b3_nslices = 0, b3_ntrip = 0, b3_stored = 0;
    DBuf<int64_t> b3ptr;
    DBuf<int32_t> b3map, b3col;
    DBuf<double> b3val;
    int nsegs = D16_SEG;      // D16 segment bases per lane: 4, or 8 when halo columns need them
    // distributed products: slices without / with ghost columns (the first
    // run while the halo exchange is in flight)
    DBuf<int32_t> s_in, s_halo;
    int64_t n_in = 0, n_halo = 0;
    // RCM-relabelled columns (FE matrices, pls.spmv_rcm): the product reads
    // xp = x[xperm] (Ctx::rcm_x) so a slice's gathers stay local
    int64_t nperm = 0;
    DBuf<int32_t> xperm;
    int64_t bytes() const {  // bytes one product streams from the matrix
        return (d16 ? stored * 10 + nslices * (64 * 4 * nsegs + 20) + 8 + nrows_mapped * 4
                    : stored * 12 + (nslices + 1) * 8) +
               b3_stored * 28 + b3_ntrip * 4 + (b3_nslices + 1) * 8 + nperm * 20;
    }
};

// Halo of a distributed matrix: columns >= nlocal are ghosts (entries owned by
// other ranks, ordered owner-major); before each product the owned entries
// other ranks need are packed and exchanged into `ghost`.
struct Halo {
    int64_t nlocal = 0, nghost = 0, nsend = 0;
    // block-global index of every local column (owned [0, nlocal), then the
    // ghosts); for a diagonal block also of every local row (host, setup only)
    std::vector<int64_t> l2g;
    DBuf<int32_t> send_idx;
    DBuf<double> sendbuf, ghost;
    std::vector<int64_t> scnt, soff, rcnt, roff;
};

struct DevCSR {
    int64_t nrows = 0, ncols = 0, nnz = 0;
    std::shared_ptr<Halo> halo;     // distributed matrices only
    DBuf<int64_t> rp;
    DBuf<int32_t> ci;
    DBuf<double> val;
    int64_t max_row = 0;
    std::unique_ptr<DevSELL> sell;  // SpMV layout (built on demand)
    int tag = 0;                    // 1: outer operator A
    bool rcm_auto = true;           // pls.spmv_rcm -1 may relabel this matrix (not AMG level operators)
};
// Build the SELL-64 copy used by every SpMV with this matrix.
void build_sell(DevCSR &M, Ctx &c);

void upload_csr(DevCSR &M, int64_t nrows, int64_t ncols, const int64_t *rp, const int32_t *ci, const double *val,
                Ctx &c);
// Extract rows [r0, r1) with a column window (see WindowSpec), columns shifted.
void extract_csr(const DevCSR &src, int64_t r0, int64_t r1, WindowSpec w, int64_t cshift, int64_t ncols,
                 DevCSR &dst, Ctx &c);
// Distributed D16 matrices: split the slices into interior / halo lists (the
// product overlaps the halo exchange with the interior slices).  build_sell
// calls it for matrices with a halo.
void classify_halo_slices(DevCSR &M, Ctx &c);
void spmv(const DevCSR &M, const double *x, double *y, Ctx &c, double alpha = 1.0, double beta = 0.0,
          const double *z = nullptr);
void spmv_slices(const DevCSR &M, const double *x, double *y, Ctx &c, double alpha, double beta, const double *z,
                 const int32_t *slist, int64_t count, size_t lds_reserve = 0);

// Host copy of a CSR matrix (setup-time algebra: fieldsplit blocks, AMG hierarchy).
// std::allocator whose value-initialisation is default-initialisation: a
// resize(n) of a host matrix array leaves it unwritten (its writer fills it,
// on as many threads as it likes) instead of zeroing GBs on one thread
// Arrays of 2 MB and more are mapped on their own with MADV_HUGEPAGE (the
// boxes run transparent huge pages in madvise mode): the setup's random
// accesses over GB-sized host matrices (the Galerkin product's P rows, the
// first pass's lambda array) otherwise miss the TLB on 4 KB pages, and a
// first touch costs one fault per 4 KB.
void *huge_alloc(size_t bytes);
void huge_free(void *p, size_t bytes);
static constexpr size_t HUGE_ALLOC_MIN = (size_t)2 << 20;
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U> &) noexcept {}
    T *allocate(size_t n) {
        if (n * sizeof(T) >= HUGE_ALLOC_MIN) return static_cast<T *>(huge_alloc(n * sizeof(T)));
        return std::allocator<T>::allocate(n);
    }
    void deallocate(T *p, size_t n) noexcept {
        if (n * sizeof(T) >= HUGE_ALLOC_MIN) huge_free(p, n * sizeof(T));
        else std::allocator<T>::deallocate(p, n);
    }
    template <class U>
    void construct(U *p) noexcept {
        ::new ((void *)p) U;
    }
    template <class U, class... Args>
    void construct(U *p, Args &&...args) {
        ::new ((void *)p) U(std::forward<Args>(args)...);
    }
};
template <class T>
using hvec = std::vector<T, NoInitAlloc<T>>;

struct HostCSR {
    int64_t nrows = 0, ncols = 0;
    hvec<int64_t> rp{0};
    hvec<int32_t> ci;
    hvec<double> v;
};
HostCSR download(const DevCSR &M, Ctx &c);
void upload(const HostCSR &H, DevCSR &M, Ctx &c);

// ----------------------------------------------------------------- options --
struct Options {
    std::map<std::string, std::string> kv;
    void parse(const char *text);
    bool has(const std::string &k) const { return kv.count(k) > 0; }
    std::string str(const std::string &k, const std::string &d) const;
    double num(const std::string &k, double d) const;
    int64_t integer(const std::string &k, int64_t d) const;
    bool flag(const std::string &k, bool d) const;
};

// -------------------------------------------------------------- timer pool --
enum TimerCat { T_PC_TOTAL = 0, T_PC_SOLID, T_PC_FLUID, T_PC_PRESS, T_PC_ALLOC, T_SOLVER, T_SPMV, T_NCAT };
struct Timers {
    double acc[T_NCAT] = {0};
    int64_t spmv_calls = 0;
    bool enabled = true;
    std::vector<hipEvent_t> pool;
    struct Pending { int cat; hipEvent_t a, b; };
    std::vector<Pending> pending;
    std::vector<int> open_stack;
    std::vector<hipEvent_t> open_ev;
    size_t next = 0;
    hipStream_t st = nullptr;
    ~Timers();
    hipEvent_t ev();
    void begin(int cat);
    void end(int cat);
    void flush();  // call after a stream sync
    void reset() { for (double &a : acc) a = 0; spmv_calls = 0; }
};

// --------------------------------------------------------------- operators --
struct Op {
    int64_t n = 0;
    virtual ~Op() = default;
    virtual void apply(const double *x, double *y, Ctx &c) = 0;
};
struct MatOp : Op {
    const DevCSR *M;
    Timers *timers = nullptr;
    explicit MatOp(const DevCSR *m) : M(m) { n = m->nrows; }
    Ctx *ctx_for_build = nullptr;
    void apply(const double *x, double *y, Ctx &c) override;
};

// --------------------------------------------------------- preconditioners --
struct PC {
    std::string type;
    int64_t n = 0;
    virtual ~PC() = default;
    virtual void apply(const double *x, double *y, Ctx &c) = 0;
    // apply() may run on two streams at once (no per-application device state)
    virtual bool reentrant() const { return false; }
};
struct PCNone : PC {
    explicit PCNone(int64_t n_) { type = "none"; n = n_; }
    bool reentrant() const override { return true; }
    void apply(const double *x, double *y, Ctx &c) override;
};
struct PCJacobi : PC {
    DBuf<double> dinv;
    PCJacobi(const DevCSR &M, Ctx &c);
    bool reentrant() const override { return true; }
    void apply(const double *x, double *y, Ctx &c) override;
};
// Level-aligned SELL-64 strict triangular factor (see kernels.hip).
struct TriSELL {
    int64_t nslices = 0, ngroups = 0, nblocks = 0;
    bool blockwise = false;
    DBuf<int64_t> sptr, gslice, goff;
    DBuf<int32_t> slot_row, slot_len, col;
    DBuf<double> val, sdinv;
    std::vector<int64_t> gslice_h;
    void apply(const double *b, double *y, Ctx &c) const;
};

// ILU(0) of the block-Jacobi truncation of M (nblocks == 1: plain ILU(0)).
// exact_lu: the same pipeline on the profile (envelope) pattern of M -- row i
// spans the contiguous columns [first nonzero of row i, max column of rows
// <= i], which contains every fill entry of LU without pivoting, so the
// "ILU" of that pattern is the exact LU factorization (PCLU).
// Factorization: level scheduled, one wave per row.  Sweeps: level-aligned
// SELL-64; with >= 64 blocks one workgroup per block walks its own levels,
// otherwise one launch per global level.
// LDS-kernel stream layout of a blockwise TriSELL (header entry per lane,
// block-local columns; levels/groups shared with the TriSELL).
struct LdsTri {
    DBuf<int64_t> sptr, gslice;  // slices differ from the TriSELL's (lanes per row); groups/goff are shared
    DBuf<int32_t> col, lpr;      // lpr: lanes per row, per block
    DBuf<double> val;
};
// Ring sweep tables of one triangle (kernels.hip, k_ilu_blocks_ring)
struct RingTri {
    DBuf<int64_t> coff, cg, cp;  // chunks per block / first level / [start, end) positions
    DBuf<int32_t> ord;           // position -> row (the triangle's level order)
    DBuf<int64_t> frp;           // far dependencies per position (CSR over b0 + p)
    DBuf<int32_t> fcol;          // ... block-local positions
    DBuf<double> fval;           // ... factor values
    int64_t nfar = 0;
};
// Chain-sweep stream of one triangle (kernels.hip, k_ilu_blocks_chain)
struct ChainTri {
    DBuf<int64_t> base, soff, nsl;  // per block: first entry, first slice, slice count
    DBuf<int32_t> sz, lpr;          // per slice: size | (8 entries per lane); per block: lanes per row
    DBuf<int32_t> col;
    DBuf<double> val;
};
// Window-sweep tables of one triangle (kernels.hip, k_ilu_blocks_window)
struct WinTri {
    DBuf<int64_t> woff;  // per window: off-window stream offsets (nwin + 1)
    // rec: per stream entry (value, block-local column) as 3 words -- one
    // 12-byte load each; tinv: per window the 64 x 64 inverse of its diagonal
    // block, column pairs [k / 2][lane][k % 2]
    DBuf<int32_t> rec;
    DBuf<double> tinv;
    int64_t nwin = 0;
};
// Super-window sweep tables of one triangle (kernels.hip, k_ilu_blocks_swin):
// blocks too long for LDS, in windows of 64 rows grouped into super-windows
// whose window inverses and near streams fit LDS (see build_swin_tri)
struct SwinTri {
    DBuf<int64_t> bsw;         // per block: first super-window (nblocks + 1), in processing order
    DBuf<int64_t> sw;          // per super-window: first window (global), windows, first row, end row (block-local)
    DBuf<int64_t> wnear, wfar;  // per window: near / far SELL offsets (nwin + 1)
    DBuf<int32_t> ncol, fcol;  // near: row - super-window's first row (LDS index); far: block-local row
    DBuf<double> nval, fval;
    DBuf<double> tinv;  // per window the packed triangle of the window inverse (2080 doubles)
    int64_t lds_bytes = 0, nwin = 0, nsw = 0;
};
struct PCILU : PC {
    int64_t nblocks = 1;
    // super-window sweep (Ctx::sweep_swin): blocks too long for LDS
    bool swin = false;
    SwinTri Lsw, Usw;
    // window sweep (Ctx::sweep_window): LDS-resident blocks in 64-row windows with
    // explicit inverses of the windows' triangles (one GEMV per window)
    bool window = false;
    bool window_ring = false;  // (the ring variant: y-resident, an LDS ring of the recent rows)
    int window_entries = 32;   // (the rows' most off-window entries: <= 16 loads 4 stream records per wave)
    int window_entries_L = 32, window_entries_U = 32;  // (per triangle: 4, 6 or 8 records per wave)
    bool window_mixed = false; // (ring variant: L by the y-resident level sweep, U by windows)
    DBuf<int64_t> zgoff;       // (no levels: the mixed sweep's empty U for the level launch)
    WinTri Lw, Uw;
    DBuf<int64_t> wstart;  // per block: its first window
    // chain sweep (Ctx::sweep_chain): LDS-resident blocks of deep, narrow level DAGs
    bool chain = false;
    ChainTri Lc, Uc;
    // ring sweep (pls.ilu_ring, default on): y-resident blocks whose levels are
    // narrow sweep in level-order position space with an LDS ring of recent values
    bool ring = false;
    RingTri Lr, Ur;
    DBuf<int32_t> mapUL;  // U position -> index of the row's L-sweep value
    std::map<hipStream_t, std::pair<DBuf<double>, DBuf<double>>> ring_scratch;  // per stream: yL, yU
    DevCSR F;                     // truncated matrix, factored in place
    DBuf<int64_t> diag;
    DBuf<double> dinv;
    TriSELL Lf, Uf;
    LdsTri Ls, Us;            // built when the LDS kernel serves apply()
    bool use_lds = false;  // one workgroup per block sweeps (k_ilu_blocks_lds)
    bool lds_gmem = false;  // ... with the block solution kept in y (blocks too long for LDS)
    int lds_tpb = 1024;     // threads per workgroup of the LDS sweep (set from the widest level; pls.sweep_tpb)
    int lds_depth = 2;      // levels of factor data in flight in the LDS sweep (pls.sweep_depth 2 / 3 / 4)
    bool lds_rr = false;    // round-robin level sweep (deep DAGs of ~one slice per level; pls.sweep_rr)
    int64_t nlev_L = 0, nlev_U = 0;
    bool allow_lds = true;  // block solution resident in LDS when it fits
    bool exact = false;     // envelope pattern: exact LU (PCLU)
    // gmem_mode -2: per-level launches straight from the factored CSR, 16 lanes
    // per row (long rows, wide levels: the AMG's Gauss-Seidel triangles)
    bool csr_levels = false;
    DBuf<int32_t> lrowsL, lrowsU;
    std::vector<int64_t> lptrL, lptrU;
    std::string profile_tag;  // non-empty: dump per-block sweep timings once (option pls.sweep_profile)
    // gmem_mode (option pls.ilu_gmem): 0 auto, 1 force the y-resident
    // workgroup sweep (also on blocks that fit LDS), -1 never, -2 never and
    // per-level CSR kernels instead of the SELL-64 level slices
    // sgs: no ILU(0) -- the factors are symmetric Gauss-Seidel's (I + L D^-1, D + U;
    // launch_sgs_factor), so apply() is one hybrid symmetric GS sweep from 0 with
    // the blocks as hypre's thread chunks (boomeramg.cpp)
    bool sgs = false;
    // explicit block starts (bounds: nblocks + 1 entries from 0 to n) instead of PETSc's bjacobi sizes
    std::vector<int64_t> bstart_h;
    DBuf<int64_t> bstart;
    int64_t max_len = 0;  // longest block
    PCILU(const DevCSR &M, int64_t nblocks, Ctx &c, bool exact_lu = false, bool allow_lds = true, int force_lpr = 0,
          int gmem_mode = 0, int ring_mode = 1, bool sgs_factors = false, const std::vector<int64_t> *bounds = nullptr);
    bool reentrant() const override { return profile_tag.empty(); }
    void apply(const double *x, double *y, Ctx &c) override;
    const char *sweep_kind() const;  // which apply kernel serves this PC (pls.ilu_view)
    // the plain LDS sweep can run a subset of its blocks (the 2-way PC's
    // pressure-first pipeline, capi.cpp BlockPC::apply): levels (L + U) and
    // first row of every block, host copies made at setup
    std::vector<int64_t> block_levels_h, block_start_h, block_maxsl_h;  // maxsl: most slices of any level
    bool can_apply_blocks() const {
        return use_lds && !ring && !window && !chain && !swin && !lds_gmem && profile_tag.empty() && !exact && !sgs;
    }
    // rr_group > 0: the round-robin sweep with groups of that many waves per level (a power of two)
    // tpb > 0: threads per workgroup for this launch; depth: levels of factor data in flight (2, or 6 with tpb <= 512)
    void apply_blocks(const double *x, double *y, Ctx &c, int64_t b_lo, int64_t b_hi, int rr_group = 0, int tpb = 0,
                      int depth = 2, int64_t *prof = nullptr);  // prof: nblocks x 8 wall-clock records (diagnostics)
};
// Exact LU of a block small enough for a dense inverse (dense.hip): K^-1 is
// formed once (blocked Gauss-Jordan, no pivoting, like the sparse path) and
// applied as one dense GEMV.  Chosen for -pc_type lu when n <= pls.lu_dense_max.
struct PCDenseLU : PC {
    int64_t ld = 0;
    DBuf<double> inv;
    DBuf<int32_t> rowperm;  // threshold pivoting's row order (empty: none); inv = (Pi M)^-1
    int32_t piv_stats[3] = {0, 0, 0};  // rows exchanged, pivots below u x column max, zero columns
    // u: MUMPS's relative pivot threshold CNTL(1) (pls.lu_pivot_threshold, default 0.01; 0 = no pivoting)
    PCDenseLU(const DevCSR &M, Ctx &c, double u = 0.0);
    bool reentrant() const override { return true; }
    void apply(const double *x, double *y, Ctx &c) override;
};
// Exact LU of a banded block past the dense-inverse size (band.hip): 64 x 64
// tiles, right-looking factorization without pivoting, flag-chained sweeps.
// Not reentrant (the sweeps share the granules, the ticket and t).
struct PCBandLU : PC {
    int64_t nb = 0, bl = 0, bu = 0;
    DBuf<double> T, Dl, Du, Gl, Gu, t;  // Gl / Gu: near-tile products (band.hip)
    DBuf<int32_t> fail;
    DBuf<uint64_t> G, ticket;  // G: 128 tagged granules per tile row (the sweeps' hand-off)
    uint64_t sweeps = 0;  // launched sweeps (ticket base = sweeps * band_sweep_tickets(nb))
    int64_t plen = 0;     // SPIKE partition length in tile rows (0: one chain per triangle)
    DBuf<double> Wl, Wu;  // SPIKE spikes of L and U (nb x bl, nb x bu tiles)
    DBuf<double> spike_tmp;  // tail partial sums
    // spike_plen: -1 auto (~16 partitions), 0 off, > 0 partition length in tile rows
    PCBandLU(const DevCSR &M, int64_t kl, int64_t ku, Ctx &c, int64_t spike_plen = -1);
    void apply(const double *x, double *y, Ctx &c) override;
    int32_t check_fail(Ctx &c);  // synchronising: the fail word (2: a sweep spin gave up)
};
// Lower / upper bandwidth of a square CSR matrix with sorted rows.
void csr_bandwidths(const DevCSR &M, int64_t &kl, int64_t &ku, Ctx &c);
// -pc_type lu / cholesky (MUMPS in the reference): dense inverse up to
// pls.lu_dense_max rows, else the sparse (nested dissection, multifrontal) LU;
// pls.lu_path dense|sparse|band|envelope forces one.
std::unique_ptr<PC> make_lu(const DevCSR &M, const Options &o, Ctx &c);
// Sparse LU by nested dissection + multifrontal factorization (sparse_lu.cpp)
std::unique_ptr<PC> make_sparse_lu(const DevCSR &M, const Options &o, Ctx &c);
void sparse_lu_analyze(const HostCSR &A, const Options &o, double *stats, int64_t nstats, int32_t *perm = nullptr,
                       int32_t *front_of = nullptr, int32_t *parent = nullptr);
std::unique_ptr<PC> make_pc(const std::string &type, const DevCSR &M, const Options &o, const std::string &prefix,
                            Ctx &c);
// Smoothed-aggregation AMG (amg.cpp; -pc_type gamg, and hypre with pls.hypre sa).
std::unique_ptr<PC> make_amg(const DevCSR &M, const Options &o, const std::string &prefix, bool hypre, Ctx &c);
// Classical AMG as the reference configures BoomerAMG (boomeramg.cpp; -pc_type hypre).
std::unique_ptr<PC> make_boomeramg(const DevCSR &M, const Options &o, const std::string &prefix, Ctx &c);
// hypre's np = G hierarchy on a sharded block (M: this rank's rows; global: the gathered block)
std::unique_ptr<PC> make_boomeramg_dist(const DevCSR &M, const HostCSR &global, const std::vector<int64_t> &rank_rows,
                                        const Options &o, const std::string &prefix, Ctx &c);
void boomeramg_host_level(const HostCSR &A, const Options &o, const std::string &prefix, int64_t level,
                          int64_t &nlevels, int64_t &n, int64_t &nc, std::vector<int8_t> &cf, HostCSR &P);

// ---------------------------------------------------------------------- KSP --
enum Reason {
    CONVERGED_ITERATING = 0, CONVERGED_RTOL = 2, CONVERGED_ATOL = 3, CONVERGED_ITS = 4,
    DIVERGED_NULL = -2, DIVERGED_ITS = -3, DIVERGED_DTOL = -4, DIVERGED_BREAKDOWN = -5,
    DIVERGED_INDEFINITE_PC = -8, DIVERGED_NANORINF = -9, DIVERGED_INDEFINITE_MAT = -10,  // petscksp.h
    DIVERGED_TIME_LIMIT = -100  // libpls diagnostic (pls.solver_time_limit), not a PETSc reason
};

struct KSP {
    std::string prefix, type = "gmres";
    double rtol = 1e-5, atol = 1e-50, dtol = 1e4;
    int64_t maxit = 10000, restart = 30;
    bool right = false;
    std::string norm = "preconditioned";
    Op *A = nullptr;
    PC *pc = nullptr;
    std::unique_ptr<PC> owned_pc;
    std::unique_ptr<Op> owned_op;
    int64_t n = 0;
    // results
    int its = 0, reason = 0;
    double rnorm = 0;
    std::vector<double> history;
    bool keep_history = true;
    bool monitor = false;
    // pls.ksp_stats: iteration totals printed when the KSP is destroyed (diagnostics)
    bool stats = false;
    double time_limit = 0;  // seconds (pls.solver_time_limit, the outer solver only; 0: none)
    double t_start = 0;
    int64_t stat_its = 0, stat_max = 0, stat_solves = 0, stat_div = 0;  // stat_div: solves with reason < 0
    int64_t stat_last_neg = 0;  // the most recent negative reason
    KSP() = default;
    KSP(const KSP &) = delete;
    ~KSP();
    // work
    DBuf<double> V, w, t1, t2, t3, t4;
    int64_t ldv = 0;  // column stride of the Krylov basis V
    DBuf<double> dh;  // device Hessenberg column / coefficients
    DBuf<double> cgS, cghist;  // device-resident CG: scalar state, residual history
    DBuf<int64_t> cgI;
    bool cg_device = true;     // pls.cg_device: CG's recurrences on the device (no read-back per iteration)
    int64_t allocated_k = -1;
    void set_type_defaults();
    void resolve_side_norm(const std::string &side, const std::string &nt);
    void solve(const double *b, double *x, Ctx &c);
    // a PREONLY solve whose PC was applied by the caller (BlockPC's fp pipeline): its bookkeeping
    void note_preonly() {
        history.clear();
        its = 1;
        reason = CONVERGED_ITS;
        stat_its += 1;
        stat_max = std::max<int64_t>(stat_max, 1);
        ++stat_solves;
    }
  private:
    void ensure_work(Ctx &c);
    void solve_gmres(const double *b, double *x, Ctx &c);
    void solve_cg(const double *b, double *x, Ctx &c);
    void solve_cg_dev(const double *b, double *x, Ctx &c);
    int converged(int it, double r);
    double rnorm0 = 0, ttol = 0;
};

// PCFIELDSPLIT with two splits given as index sets of the matrix rows
// (reference lib/Preconditioner.py:102-118: split 0 = is_p, split 1 = is_f in
// fp-local numbering).  Types additive, multiplicative, schur (fact diag /
// lower / upper / full; Schur preconditioning matrix selfp or a11; Schur KSP
// operator S = A11 - A10 A00^-1 A01 applied implicitly with the split-0 KSP).
struct PCFieldSplit : PC {
    std::string ftype, fact;
    double scale = -1.0;
    int64_t n0 = 0, n1 = 0;
    DBuf<int32_t> is0, is1;
    DevCSR A00, A01, A10, A11, Sp;
    std::unique_ptr<KSP> k0, k1;
    DBuf<double> x0, x1, y0, y1, t0, t1;
    PCFieldSplit(const DevCSR &M, const std::vector<int32_t> &is0, const std::vector<int32_t> &is1, const Options &o,
                 const std::string &prefix, Ctx &c);
    void apply(const double *x, double *y, Ctx &c) override;
};

// PCREDUNDANT: a sharded diagonal block (Halo::l2g) gathered on every rank,
// factory(global block, single-rank context) builds the PC applied redundantly.
// Sharded diagonal block -> the global host CSR on every rank (PCRedundant's
// gather; rank_rows: the ranks' row counts when contiguous in rank order)
HostCSR gather_block(const DevCSR &M, Ctx &c, const std::string &prefix, std::vector<int64_t> &srcslot,
                     int64_t &maxloc, std::vector<int64_t> &rank_rows);
// a single-rank context with c's layout options (own stream)
std::unique_ptr<Ctx> layout_ctx(const Ctx &c);
// local rows with global columns owned in contiguous rank ranges cst -> distributed DevCSR with halo
void upload_dist(const HostCSR &L, const std::vector<int64_t> &cst, DevCSR &M, Ctx &c);
// (a block gather_block already produced, consumed by make_redundant instead of gathering again)
struct GatheredBlock {
    HostCSR G;
    std::vector<int64_t> srcslot, rank_rows;
    int64_t maxloc = 0;
};
std::unique_ptr<PC> make_redundant(const std::string &type, const DevCSR &M, Ctx &c,
                                   const std::function<std::unique_ptr<PC>(const DevCSR &, Ctx &)> &factory,
                                   const std::string &prefix, GatheredBlock *pre = nullptr);
// Configure a KSP from programmatic defaults + options (setFromOptions order).
std::unique_ptr<KSP> make_ksp(const std::string &prefix, const Options &o, const DevCSR *Amat, const DevCSR *Pmat,
                              const std::string &default_ksp, const std::string &default_pc, Ctx &c,
                              double rtol = 1e-5, double atol = 1e-50, double dtol = 1e4, int64_t maxit = 10000,
                              int64_t restart = 30, PC *external_pc = nullptr);

}  // namespace pls
