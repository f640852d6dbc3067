// kernels.hpp -- host launchers of the HIP/CDNA4 kernels (kernels.hip).
// Every launcher enqueues on `st` and never synchronises.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace pls {

// ----------------------------------------------------------------- synth --
struct SynthDev {
    int32_t dim;
    uint64_t seed;
    double delta;
    int64_t n[3];
    int64_t off[3];
    int32_t cnt[6];
    const int32_t *offs[6];  // device pointers, sorted offsets per forward block
    // rows generated: local row l in [rloff[f], rloff[f] + rlen[f]) is global
    // row off[f] + rlo[f] + (l - rloff[f]) (identity for a single rank)
    int64_t rlo[3], rlen[3], rloff[3], nrows;
};
void launch_synth_count(const SynthDev &S, int64_t *row_len, hipStream_t st);
void launch_synth_fill(const SynthDev &S, int variant, const int64_t *row_ptr, int32_t *col,
                       double *val, hipStream_t st);
void launch_synth_rhs(const SynthDev &S, uint64_t seed, double *b, hipStream_t st);

// ---------------------------------------------------------------- CSR ops --
// Exclusive scan of n+1 entries: in[0..n) lengths -> out[0..n] offsets.
void exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n, void *tmp, size_t tmp_bytes,
                        hipStream_t st);
size_t exclusive_scan_tmp_bytes(int64_t n);

// Column-window extraction: rows [r0, r1) of (rp, ci, val); keep entries with
// column in the window of the row; output columns shifted by -cshift.
//   mode 0: window [c0, c1) for every row
//   mode 1: block-Jacobi window of the row's block, blocks over [0, r1-r0)
//           with PETSc sizes (first nb % .. blocks one longer), cshift = r0
struct WindowSpec {
    int mode;
    int64_t c0, c1;
    int64_t nblocks;                  // mode 1
    const int64_t *bstart = nullptr;  // mode 1: explicit block starts (nblocks + 1, device), else PETSc sizes
};
void launch_extract_count(const int64_t *rp, const int32_t *ci, int64_t r0, int64_t r1,
                          WindowSpec w, int64_t *row_len, hipStream_t st);
void launch_extract_fill(const int64_t *rp, const int32_t *ci, const double *val, int64_t r0,
                         int64_t r1, WindowSpec w, int64_t cshift, const int64_t *out_rp,
                         int32_t *out_ci, double *out_val, hipStream_t st);

// y = alpha * (M x) + beta * z     (z may be null when beta == 0)
void set_spmv_short_rows(bool on);  // CSR rows of < 12 entries: one lane per row (default off; pls.spmv_short 1, opt-in)
void launch_spmv(int64_t nrows, int64_t nnz, const int64_t *rp, const int32_t *ci,
                 const double *val, const double *x, double *y, double alpha, double beta,
                 const double *z, hipStream_t st);

// ----------------------------------------------------------------- BLAS-1 --
void launch_copy(int64_t n, const double *x, double *y, hipStream_t st);
void launch_copy_probe(int64_t n, const double *x, double *y, int mode /*0 copy, 1 read*/, hipStream_t st);
void launch_set(int64_t n, double a, double *y, hipStream_t st);
void launch_scale(int64_t n, double a, double *y, hipStream_t st);
// y = a*x + b*y
void launch_axpby(int64_t n, double a, const double *x, double b, double *y, hipStream_t st);
// the same with a = *pa, b = *pb read on the device; a no-op when *skip (device-resident CG)
void launch_axpby_dev(int64_t n, const double *pa, const double *x, const double *pb, double *y, const int64_t *skip,
                      hipStream_t st);
// device-resident CG (KSP::solve_cg_dev): scalar state S (doubles) / I (ints) and its phases
enum CgS { CG_BETA, CG_BETAOLD, CG_DPI, CG_A, CG_NEGA, CG_BB, CG_ONE, CG_RNORM, CG_RNORM0, CG_TTOL, CG_SLOT, CG_SLOT2,
           CG_NS = 16 };
enum CgI { CG_DONE, CG_ITS, CG_REASON, CG_HCOUNT, CG_NI = 8 };
enum CgPhase { CG_TOP, CG_MID, CG_POST, CG_END };
struct CgParams {
    double rtol, atol, dtol;
    int64_t maxit;
    int norm;  // 0 none, else the norm of S[CG_SLOT] is the residual norm
    int r_rtol, r_atol, r_dtol, r_nan, r_its, r_indef_pc, r_indef_mat;  // the KSPConvergedReason codes
};
void launch_cg_state(int phase, int64_t i, double *S, int64_t *I, double *hist, const CgParams &p, hipStream_t st);
// w = a*x + b*y  (out of place)
void launch_waxpby(int64_t n, double a, const double *x, double b, const double *y, double *w,
                   hipStream_t st);
void launch_pointwise_mult(int64_t n, const double *x, const double *d, double *y, hipStream_t st);
// AMG smoother step: d = a d + bc (dinv . r); x += d.  flags 1: d not read
// (d = bc (dinv . r)); flags 2: x not read (x = d)
void launch_cheb_step(int64_t n, const double *dinv, const double *r, double *d, double *x, double a, double bc,
                      int flags, hipStream_t st);
void launch_zero_entries(int64_t m, const int32_t *idx, double *y, hipStream_t st);
void launch_gather(int64_t n, const int64_t *idx, const double *x, double *y, hipStream_t st);
void launch_scatter(int64_t n, const int64_t *idx, const double *x, double *y, hipStream_t st);

// deterministic reductions: fixed grid (depends only on n)
int reduce_blocks(int64_t n);
// partial[j*NB + b] for j < k :  dot(v_j, w) ; then final into out[j]
void launch_mdot(int64_t n, int k, const double *const *v_dev_ptrs, const double *V, int64_t ldv,
                 const double *w, double *partial, double *out, hipStream_t st);
void launch_dot(int64_t n, const double *x, const double *y, double *partial, double *out,
                hipStream_t st);
// out = ||x||_2 (sqrt of sum of squares)
void launch_norm2(int64_t n, const double *x, double *partial, double *out, hipStream_t st);
// w -= sum_j h[j] * V[:, j] (h on device, j < k); out = ||w||_2^2 (local) when out != null
void launch_maxpy_norm(int64_t n, int k, const double *V, int64_t ldv, const double *h_dev,
                       double hscale, double *w, double *partial, double *out, hipStream_t st);
// y = sum_j c[j] * V[:, j] (c on device)
void launch_lincomb(int64_t n, int k, const double *V, int64_t ldv, const double *c_dev, double *y,
                    hipStream_t st);
// TSQR step (Anderson least squares): R of each TSQR rows-per-block row chunk of the
// m <= 16 columns, written as rows [b m, b m + m) of a column-major matrix (leading dim ldo)
int tsqr_rows_per_block();
void launch_tsqr(int64_t n, int m, const double *const *cols_dev, double *Rout, int64_t ldo, hipStream_t st);

// -------------------------------------------------------------------- ILU --
// Factor the rows of one level in place (original CSR): lu, diag pos, dinv.
// max_row: longest row of the matrix (<= ilu0_max_row(); staged in LDS).
int ilu0_max_row();
// max_staged: the most upper-part entries of one row's pivots (LDS sizing)
void launch_ilu0_level(int64_t nrows_level, const int32_t *rows, const int64_t *rp,
                       const int32_t *ci, double *lu, const int64_t *diag, double *dinv,
                       int32_t *fail, int64_t max_row, int64_t max_staged, hipStream_t st);
// all levels in one launch (rows in level order; done: n flags, ctr: 2 ints -- scratch)
void launch_ilu0_dep(int64_t n, const int32_t *rows, const int64_t *rp, const int32_t *ci, double *lu,
                     const int64_t *diag, double *dinv, int32_t *fail, int64_t max_row, int64_t max_staged,
                     int32_t *done, int32_t *ctr, hipStream_t st);
// test knobs (process-wide; pls.ilu0_stage, pls.ilu_dep_grid): stage_cap < 0 default,
// 0 no staged pivots, > 0 at most that many staged entries; grid_cap > 0 caps
// k_ilu0_dep's persistent grid (1: one workgroup)
void set_ilu0_test_caps(int stage_cap, int grid_cap);
void launch_find_diag(int64_t n, const int64_t *rp, const int32_t *ci, int64_t *diag, int32_t *fail,
                      hipStream_t st);
// Symmetric Gauss-Seidel "factors" in ILU(0) storage (hypre relax type 6 as a
// preconditioner M = (D + L) D^-1 (D + U)): strict-lower entries scaled by the
// column's 1/a_jj (the unit lower factor I + L D^-1), diagonal and upper kept
// (the upper factor D + U), dinv = 1/a_ii; fail |= 2 on a zero diagonal.
void launch_sgs_factor(int64_t n, const int64_t *rp, const int32_t *ci, double *lu, const int64_t *diag,
                       double *dinv, int32_t *fail, hipStream_t st);
// Level-ordered triangular factor storage ("row r of level order"): build
void launch_lvl_count(int64_t n, const int32_t *order, const int64_t *rp, const int64_t *diag,
                      int upper, int64_t *len, hipStream_t st);
void launch_lvl_fill(int64_t n, const int32_t *order, const int64_t *rp, const int32_t *ci,
                     const double *lu, const int64_t *diag, int upper, const int64_t *out_rp,
                     int32_t *out_ci, double *out_val, hipStream_t st);
// One level of the forward (unit lower) sweep: y[i] = b[i] - sum l_ij y[j]
// One level of the backward sweep:           y[i] = (y[i] - sum u_ij y[j]) * dinv[i]
void launch_trsv_level(int64_t r0, int64_t r1, const int32_t *row_of, const int64_t *rp,
                       const int32_t *ci, const double *val, const double *dinv_lvl,
                       const double *b, double *y, int lanes_per_row, hipStream_t st);

// Block-Jacobi sweep: blocks independent, one workgroup per block.
// blk_off[b]..blk_off[b+1] index lvl_ptr (row boundaries of block b's levels).
void launch_trsv_blocks(int64_t nblocks, const int64_t *blk_off, const int64_t *lvl_ptr, const int32_t *row_of,
                        const int64_t *rp, const int32_t *ci, const double *val, const double *dinv_lvl,
                        const double *b, double *y, int lanes_per_row, hipStream_t st);

// SELL-64 (sliced ELLPACK, slice = 64 rows = one wave)
int64_t sell_nslices(int64_t nrows);
void launch_sell_slice_len(int64_t nrows, const int64_t *rp, int64_t *slen /* nslices+1 */, hipStream_t st);
void launch_sell_fill(int64_t nrows, const int64_t *rp, const int32_t *ci, const double *val, const int64_t *sptr,
                      int32_t *scol, double *sval, hipStream_t st);
// tag 1 = the outer operator A (separate kernel symbol in profiles);
// ghost != null: columns >= nlocal read ghost[c - nlocal] (halo entries)
void launch_sell_spmv(int64_t nrows, const int64_t *sptr, const int32_t *scol, const double *sval, const double *x,
                      double *y, double alpha, double beta, const double *z, int tag, const double *ghost,
                      int64_t nlocal, hipStream_t st);
// SELL-64 / D16 (16-bit column deltas, D16_SEG segment bases per lane, 1 or 8 lanes per row)
constexpr int D16_SEG = 4;      // segment bases per lane (rows of a single rank)
constexpr int D16_SEG_MAX = 8;  // ... with halo columns (own s/f/p + a neighbour's s/f/p)
void launch_d16_slice_len(int64_t nslices, const int64_t *sfirst, const int32_t *slpr, const int64_t *rp,
                          int64_t nrows, int64_t *slen /* nslices+1 */, hipStream_t st,
                          const int32_t *rowmap = nullptr /* slice position -> row (SELL-C-sigma) */);
void launch_d16_count(int64_t nslices, const int64_t *sfirst, const int32_t *slpr, const int64_t *rp,
                      const int32_t *ci, int64_t nrows, int32_t *maxseg, hipStream_t st,
                      const int32_t *rowmap = nullptr);
void launch_d16_fill(int64_t nslices, const int64_t *sfirst, const int32_t *slpr, const int64_t *rp,
                     const int32_t *ci, const double *val, int64_t nrows, const int64_t *sptr, uint16_t *dl,
                     double *dv, int32_t *seg, int nsegs /* D16_SEG or D16_SEG_MAX */, hipStream_t st,
                     const int32_t *rowmap = nullptr);
void launch_first_col(int64_t nrows, const int64_t *rp, const int32_t *ci, int32_t *c0, hipStream_t st);
void launch_d16_spmv(int64_t nrows, int64_t nslices, const int64_t *sptr, const int64_t *sfirst, const int32_t *slpr,
                     const uint16_t *dl, const double *dv, const int32_t *seg, int nsegs, const double *x, double *y,
                     double alpha, double beta, const double *z, int tag, const double *ghost, int64_t nlocal,
                     int unroll /* 8-entry groups per lane in flight: 1, 2 or 4 */, hipStream_t st,
                     const int32_t *slist = nullptr /* nslices entries: the slices to process */,
                     const int32_t *rowmap = nullptr /* slice position -> row (SELL-C-sigma) */,
                     size_t lds_reserve = 0 /* dynamic LDS per workgroup, unused: keeps the product's
                                               workgroups off CUs whose LDS a sweep holds */);
// SELL/B3: row triples sharing one column list (FE vector fields), see kernels.hip
void launch_triple_flags(int64_t n, const int64_t *rp, const int32_t *ci, uint8_t *flag, hipStream_t st);
int b3_lanes_per_triple();
void launch_b3_fill(int64_t nslices, int64_t ntrip, const int64_t *bptr, const int32_t *tmap, const int64_t *rp,
                    const int32_t *ci, const double *val, int32_t *bcol, double *bval, hipStream_t st);
void launch_b3_spmv(int64_t nslices, int64_t ntrip, const int64_t *bptr, const int32_t *tmap, const int32_t *bcol,
                    const double *bval, const double *x, double *y, double alpha, double beta, const double *z,
                    int tag, hipStream_t st);
// D16 SpMV workgroup -> slice order: 0 round-robin over the 8 XCDs (default), 1 XCD-contiguous ranges
void set_d16_xcd(int on);
// flag[r] = 1 when row r (sorted columns) references a ghost column (>= nlocal)
void launch_row_has_ghost(int64_t nrows, const int64_t *rp, const int32_t *ci, int64_t nlocal, uint8_t *flag,
                          hipStream_t st);

// Level-aligned SELL-64 triangular factors (see kernels.hip)
void launch_tri_fill(int64_t nslices, const int32_t *slot_row, const int32_t *slot_len, const int64_t *rp,
                     const int32_t *ci, const double *lu, const int64_t *diag, const double *dinv, int upper,
                     const int64_t *sptr, int32_t *ocol, double *oval, double *odinv, hipStream_t st);
void launch_tri_blocks(int64_t nblocks, const int64_t *goff, const int64_t *gslice, const int64_t *sptr,
                       const int32_t *slot_row, const int32_t *slot_len, const int32_t *col, const double *val,
                       const double *sdinv, const double *b, double *y, hipStream_t st);
// one level of a triangular sweep from the factored CSR, 16 lanes per row (kernels.hip)
void launch_tri_csr_level(int64_t m, const int32_t *rows, const int64_t *rp, const int32_t *ci, const double *val,
                          const int64_t *diag, const double *dinv, int upper, const double *b, double *y,
                          hipStream_t st);
void launch_tri_group(int64_t s0, int64_t s1, const int64_t *sptr, const int32_t *slot_row, const int32_t *slot_len,
                      const int32_t *col, const double *val, const double *sdinv, const double *b, double *y,
                      hipStream_t st);

// Block-Jacobi ILU(0) apply, one workgroup per block, levels separated by
// workgroup barriers (forward + backward in one launch).  Block solution
// resident in LDS when every block has <= ilu_lds_max_rows() rows; gmem: kept
// in y instead (blocks of up to ilu_gmem_max_rows() rows).
int ilu_lds_max_rows();
int ilu_gmem_max_rows();
void launch_ilu_blocks_lds(int64_t n, int64_t nblocks, const int64_t *Lgoff, const int64_t *Lgslice,
                           const int64_t *Lsptr, const int32_t *Lcol, const double *Lval, const int32_t *Llpr,
                           const int64_t *Ugoff, const int64_t *Ugslice, const int64_t *Usptr, const int32_t *Ucol,
                           const double *Uval, const int32_t *Ulpr, const double *x, double *y, hipStream_t st,
                           int64_t *prof = nullptr, bool gmem = false, int tpb = 1024, int rr = 0,
                           const int64_t *bstart = nullptr, int64_t max_len = 0, int64_t blk_lo = 0,
                           int64_t blk_hi = -1,  // blocks [blk_lo, blk_hi) only (blk_hi < 0: all)
                           int depth = 2);       // levels in flight: 2, or 6 with tpb <= 512

int ilu_lds_lane_entries();
// super-window sweep (blocks too long for LDS): see kernels.hip
void launch_ilu_blocks_swin(int64_t n, int64_t nblocks, const int64_t *bstart, const int64_t *wstart,
                            const int64_t *Lbsw, const int64_t *Lsw, const int64_t *Lwnear, const int32_t *Lncol,
                            const double *Lnval, const int64_t *Lwfar, const int32_t *Lfcol, const double *Lfval,
                            const double *Ltinv, const int64_t *Ubsw, const int64_t *Usw, const int64_t *Uwnear,
                            const int32_t *Uncol, const double *Unval, const int64_t *Uwfar, const int32_t *Ufcol,
                            const double *Ufval, const double *Utinv, const double *x, double *y, int64_t lds_bytes,
                            hipStream_t st);
int ilu_swin_lds_budget();  // bytes of LDS a super-window's staged inverses + near streams may take
// The chain sweep (kernels.hip, k_ilu_blocks_chain): one wave per LDS-resident
// block walks its slices in order with ilu_chain_depth() slices in flight
// (deep, narrow level DAGs).  Per triangle and block: first slice's entry
// (base), its first slice in the size array sz (soff), the slice count (nsl),
// lanes per row (lpr, 1..ilu_chain_max_lpr()).
int ilu_chain_depth();
int ilu_chain_max_lpr();
void launch_ilu_blocks_chain(int64_t n, int64_t nblocks, const int64_t *bstart, const int64_t *Lbase,
                             const int64_t *Lsoff, const int32_t *Lsz, const int64_t *Lnsl, const int32_t *Llpr,
                             const int32_t *Lcol, const double *Lval, const int64_t *Ubase, const int64_t *Usoff,
                             const int32_t *Usz, const int64_t *Unsl, const int32_t *Ulpr, const int32_t *Ucol,
                             const double *Uval, const double *x, double *y, int64_t max_len, hipStream_t st);
// The window sweep (kernels.hip, k_ilu_blocks_window): LDS-resident blocks in
// windows of 64 rows; per block its first window wstart[b] (nblocks + 1); per
// triangle and window the off-window stream [woff[w], woff[w + 1]) ([k][lane]
// SELL of 12-byte records: value, block-local column) and the window's
// inverse in column pairs,
// tinv[w * 4096 + (k / 2) * 128 + lane * 2 + k % 2].
// The record streams carry ilu_window_stream_pad() entries of padding at
// their end (the staging copies read a fixed count); blocks of at most
// ilu_window_max_rows() rows.
int ilu_window_max_rows();
int ilu_window_stream_pad();
int ilu_window_max_entries();  // off-window entries per row the kernel handles
// The ring variant (ring = true): blocks longer than LDS, up to
// ilu_window_ring_max_rows() rows, y as the block solution and an LDS ring of
// ilu_window_ring_rows() rows for the off-window terms -- no row may depend on
// one more than ilu_window_ring_rows() - 64 rows away (the caller checks)
int ilu_window_ring_rows();
int64_t ilu_window_ring_max_rows();
void launch_ilu_blocks_window(int64_t n, int64_t nblocks, const int64_t *bstart, const int64_t *wstart,
                              const int64_t *Lwoff, const int32_t *Lrec, const double *Ltinv, const int64_t *Uwoff,
                              const int32_t *Urec, const double *Utinv, const double *x, double *y, int64_t max_len,
                              hipStream_t st, int depth = 2, bool ring = false, int tri = 3,
                              int max_entries_L = 32, int max_entries_U = 32);  // (rows' most off-window entries)
int window_records(int max_entries);  // stream records per wave and window (4, 6, 8) for that many entries
// (depth: windows of data in flight, 2 or 3; pls.window_depth; the ring variant: 2;
// tri (ring variant): 1 the L sweep, 2 the U sweep on y (holding L's solution), 3 both)
// The ring sweep (kernels.hip, k_ilu_blocks_ring): blocks of narrow levels whose
// every level has <= ilu_ring_chunk() rows; per triangle chunk tables (coff per
// block, cg first level, cp [start, end) positions), level orders ordL / ordU
// (position -> row), mapUL (U position -> yL index), scratch yL / yU (n each).
int ilu_ring_slots();
int ilu_ring_lane_entries();  // factor entries per lane per pipeline slot of the ring sweep
void set_ilu0_probe(int v);  // diagnostics only (pls.ilu0_probe)
void set_ring_probe(int v);  // diagnostics only (pls.ring_probe)
int ilu_ring_chunk();
void launch_ilu_blocks_ring(int64_t n, int64_t nblocks, const int64_t *Lgoff, const int64_t *Lgslice,
                            const int64_t *Lsptr, const int32_t *Lcol, const double *Lval, const int32_t *Llpr,
                            const int64_t *Ugoff, const int64_t *Ugslice, const int64_t *Usptr, const int32_t *Ucol,
                            const double *Uval, const int32_t *Ulpr, const int64_t *Lcoff, const int64_t *Lcg,
                            const int64_t *Lcp, const int64_t *Ucoff, const int64_t *Ucg, const int64_t *Ucp,
                            const int32_t *ordL, const int32_t *mapUL, const int32_t *ordU, const int64_t *Lfrp,
                            const int32_t *Lfcol, const double *Lfval, const int64_t *Ufrp, const int32_t *Ufcol,
                            const double *Ufval, const double *x, double *y, double *yL, double *yU, hipStream_t st, int tpb = 1024, const int64_t *bstart = nullptr);
// LDS-kernel stream layout (header entry per lane, lanes-per-row slices, block-local columns)
void launch_lds_fill(int64_t nslices, const int32_t *s_start, const int32_t *s_n, const int32_t *s_lpr,
                     const int32_t *order, const int64_t *rp, const int32_t *ci, const double *lu, const int64_t *diag,
                     const double *dinv, int upper, int64_t n, int64_t nb, const int64_t *sptr2, int32_t *ocol,
                     double *oval, hipStream_t st, bool wide = false,
                     const int32_t *posof = nullptr /* ring sweep: row -> block-local level-order position */,
                     const int32_t *row_lo = nullptr /* ring sweep: entries with position < row_lo[row] are far */, const int64_t *bstart = nullptr);

// distribution helpers
void launch_flag_ghosts(int64_t nnz, const int32_t *ci, const int32_t *own, uint8_t *flag, hipStream_t st);
void launch_remap_cols(int64_t nnz, int32_t *ci, const int32_t *gmap, hipStream_t st);
void launch_sort_rows(int64_t n, const int64_t *rp, int32_t *ci, double *val, hipStream_t st);
void launch_pack(int64_t m, const int32_t *idx, const double *x, double *buf, hipStream_t st);   // buf[k] = x[idx[k]]
void launch_unpack(int64_t m, const int32_t *idx, const double *buf, double *x, hipStream_t st); // x[idx[k]] = buf[k]

// ------------------------------------------------- dense exact LU (dense.hip) --
// M: ld x ld row-major (ld = 64 * ceil(n / 64)); pads are identity rows.
void launch_dense_from_csr(int64_t n, int64_t ld, const int64_t *rp, const int32_t *ci, const double *val, double *M,
                           hipStream_t st);
// In place M := M^-1 by blocked Gauss-Jordan; D: 64 x 64 scratch; *fail |= 1 on
// a zero pivot.  With u > 0 and P (n x 64 scratch) each tile column's pivots are
// chosen over rows [64 k, n) by threshold partial pivoting (MUMPS CNTL(1) = u;
// P then holds n x 64 + panel_fast_doubles(): the panel and the fast path's scratch),
// the rows exchanged in M and rowperm (initialised to the identity): M := (Pi M)^-1;
// stats[3] as launch_mf_panel_pivot.  u = 0: no pivoting (rounds 1-5).
void launch_dense_invert(int64_t ld, double *M, double *D, int32_t *fail, hipStream_t st, int64_t n = 0,
                         double *P = nullptr, int32_t *rowperm = nullptr, int32_t *stats = nullptr, double u = 0.0);
// y = M[:n, :n] x  (rowperm: y = M xp, xp[c] = x[rowperm[c]])
void launch_dense_gemv(int64_t n, int64_t ld, const double *M, const double *x, double *y, hipStream_t st,
                       const int32_t *rowperm = nullptr);
// Block-diagonal dense operators (hybrid Gauss-Seidel chunks of the AMG): chunk
// c holds rows [cptr[c], cptr[c+1]) and its ld x ld row-major block at
// M + c ld^2; cof[i] = chunk of row i.  y = blockdiag(M_c) x.
void launch_bdense_gemv(int64_t n, int64_t ld, const int32_t *cof, const int64_t *cptr, const double *M,
                        const double *x, double *y, hipStream_t st);
// rows r < n of the ld x ld block M scaled by d[r]
void launch_dense_rowscale(int64_t n, int64_t ld, const double *d, double *M, hipStream_t st);
// C = A B, all ld x ld row-major (ld a multiple of 64)
void launch_dense_gemm(int64_t ld, const double *A, const double *B, double *C, hipStream_t st);

// ------------------------------------------- multifrontal LU (dense.hip) --
// Frontal matrices of one level of the assembly tree (sparse_lu.cpp): front f
// is a dense ld x ld row-major block (ld = 64 ldt) at W + ws; its first p rows /
// columns are the pivots (padded to 64 pt), the rest the update rows (q real).
struct MFront {
    int64_t ws;
    int32_t ldt, pt, p, q;
};
// identity on the padding pivots [p, 64 pt) of every front
void launch_mf_pad(int nf, const MFront *F, int max_pad, double *W, hipStream_t st);
// W[dst[k]] = val[src[k]] (original entries into their fronts)
void launch_mf_scatter(int64_t m, const int64_t *dst, const int64_t *src, const double *val, double *W,
                       hipStream_t st);
// Extend-add of children's update blocks into their parents (one child per
// parent per launch, so no two children of a parent race).
struct MChild {
    int64_t src_ws, dst_ws, map_off;
    int32_t src_ld, src_pp, dst_ld, q;
};
void launch_mf_extend(int nc, const MChild *C, int max_q, const int32_t *maps, const double *Wprev, double *Wcur,
                      hipStream_t st);
// Step k of the partial Gauss-Jordan elimination of every front's pivot tiles
// (front := [F11^-1, F11^-1 F12; -F21 F11^-1, F22 - F21 F11^-1 F12]); D: nf
// 64 x 64 scratch tiles.  A pivot of magnitude <= tau (after partial pivoting
// inside the tile) is replaced by +-tau and counted in fail[1] (static
// pivoting); with tau = 0 an exact zero pivot sets fail[0] instead.
void launch_mf_gj_step(int nf, const MFront *F, int max_ldt, int k, double *W, double *D, int32_t *fail,
                       double tau, hipStream_t st);
// Threshold partial pivoting (MUMPS CNTL(1) = u) before step k: front f's tile-k
// pivots chosen among its fully-summed rows [64 k, p) (update rows the threshold's
// reference), rows exchanged in W and in rowperm + pst[f] (front-local original
// row per position); P + soff[f]: (p + q) x 64 scratch.  stats: [0] rows
// exchanged, [1] pivots below u x column max (MUMPS would delay them; dflag + pst[f]:
// 1 at those columns), [2] zero columns.  S (nf x panel_fast_doubles() scratch;
// max_rows >= every front's p + q): the parallel fast path for panels that keep
// every diagonal pivot (dense.hip k_panel_tile / k_panel_rows); the one-workgroup
// panel runs only where it does not hold.
void launch_mf_panel_pivot(int nf, const MFront *F, const int64_t *pst, const int64_t *soff, int k, double *W,
                           double *P, int32_t *rowperm, int32_t *stats, double u, hipStream_t st,
                           int32_t *dflag = nullptr, double *S = nullptr, int64_t max_rows = 0);
int panel_fast_doubles();
// Persistent factors: rows [0, 64 pt) of the front (U part, ld wide) to U + uoff
// and rows [64 pt, 64 pt + q) x columns [0, 64 pt) (X part) to X + xoff.
struct MStore {
    int64_t uoff, xoff;
};
void launch_mf_store(int nf, const MFront *F, const MStore *S, int max_rows, const double *W, double *U, double *X,
                     hipStream_t st);
// Solve (ND order).  Per front: pivots at z/x[pstart, +p), update rows = slist[soff, +q).
struct MSolve {
    int64_t pstart, qoff, uoff, xoff, soff;
    int32_t p, q, pp, ld;
};
// forward, gather: level row k = (front rf[k], local row rl[k]); v = b (pivot rows) +
// the children's contributions cu[cidx[cptr[k] ..]]; pivot rows -> z, update rows -> acc
void launch_mf_fwd_gather(int64_t m, const int32_t *rf, const int32_t *rl, const MSolve *S, const int64_t *cptr,
                          const int64_t *cidx, const double *b, const double *cu, double *z, double *acc,
                          hipStream_t st);
// forward, update rows: cu = acc + X z_p (one wave per row)
void launch_mf_fwd_gemv(int64_t m, const int32_t *rf, const int32_t *rl, const MSolve *S, const double *X,
                        const double *z, const double *acc, double *cu, hipStream_t st);
// backward, pivot rows: x_p = F11^-1 z_p - G12 x(slist) (one wave per row)
void launch_mf_bwd(int64_t m, const int32_t *rf, const int32_t *rl, const MSolve *S, const double *U,
                   const int32_t *slist, const double *z, double *x, hipStream_t st);
// y[perm[i]] = x[i] / x[i] = b[perm[i]]
void launch_gather_i32(int64_t n, const int32_t *perm, const double *b, double *x, hipStream_t st);
void launch_scatter_i32(int64_t n, const int32_t *perm, const double *x, double *y, hipStream_t st);

// ------------------------------------------------- banded exact LU (band.hip) --
// T: nb tile rows x (bl + bu + 1) tiles of 64 x 64 (see band.hip); padding
// rows past n are identity rows.
void launch_band_from_csr(int64_t n, int64_t nb, int64_t bl, int64_t bu, const int64_t *rp, const int32_t *ci,
                          const double *val, double *T, hipStream_t st);
// In place LU without pivoting; Dl / Du: nb inverted diagonal triangles;
// Gl[I] = Dl_I L_{I,I-1}, Gu[I] = Du_I U_{I,I+1} (the sweeps' near tiles);
// *fail |= 1 on a zero pivot.
void launch_band_factor(int64_t nb, int64_t bl, int64_t bu, double *T, double *Dl, double *Du, double *Gl,
                        double *Gu, int32_t *fail, hipStream_t st);
// One triangular sweep (upper 0: L with Dl, Gl; 1: U with Du, Gu), y != b.
// Gr: 128 tagged granules per tile row (zeroed once); epoch: fresh per sweep,
// never 0; ticket_base: tickets drawn by earlier sweeps (band_sweep_tickets
// per sweep) on `ticket`; *fail |= 2 if a spin gave up.
int64_t band_sweep_tickets(int64_t nb);
void launch_band_sweep(int64_t n, int64_t nb, int64_t bl, int64_t bu, const double *T, const double *Dinv,
                       const double *Gn, const double *b, double *y, uint64_t *Gr, uint64_t *ticket,
                       uint64_t ticket_base, uint32_t epoch, int upper, int32_t *fail, hipStream_t st, int64_t plen = 0);
// SPIKE partitioned sweeps (band.hip): spikes W (nb x bw tiles) of a triangle
// (upper = 0: L / Dl, bw = bl; 1: U / Du, bw = bu) for partitions of plen
// positions; apply = the corrections after a launch_band_sweep(..., plen).
void launch_spike_setup(int64_t nb, int64_t bl, int64_t bu, int upper, int64_t plen, const double *T,
                        const double *Dinv, double *Wt, hipStream_t st);
void launch_spike_apply(int64_t n, int64_t nb, int64_t bw, int upper, int64_t plen, const double *Wt, double *y,
                        double *scratch, hipStream_t st);
int64_t spike_scratch_doubles(int64_t bw);  // scratch of launch_spike_apply

}  // namespace pls
