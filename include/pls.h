/*
 * pls.h -- C-ABI of the MI355X-native block-preconditioned Krylov solver
 * ("pls" = poroelastic linear solver).  Plain pointers and sizes, no torch or
 * PETSc types.  Every entry point returns 0 on success and a nonzero status on
 * failure; pls_last_error() then returns a thread-local message (the Python
 * facade raises RuntimeError with it).
 *
 * Which reference interface each entry point replaces (reference = the
 * nabw/poroelasticity-linear-solvers tree):
 *
 *   pls_create          Preconditioner(index_map, A, P, P_diff, parameters,
 *                       bcs_sub_pressure)      lib/Preconditioner.py:263-276
 *                       + Solver(A, b, PC, parameters, index_map)
 *                                               lib/Solver.py:54-62
 *                       + IndexSet contract     lib/IndexSet.py:29-67
 *   pls_setup           Preconditioner.get_pc() -> PreconditionerCC.setUp
 *                                               lib/Preconditioner.py:120-139,282-291
 *                       + Solver.create_solver  lib/Solver.py:64-103
 *   pls_pc_apply        PreconditionerCC.apply(pc, x, y)
 *                                               lib/Preconditioner.py:141-250
 *   pls_solve           Solver.solve(b, x) -> KSPSolve / AAR.solve
 *                                               lib/Solver.py:148-152, lib/AAR.py:46-128
 *   pls_get_result      Solver.getIterationNumber / KSPGetConvergedReason /
 *                       residual history        lib/Solver.py:145-146
 *   pls_get_timings     PreconditionerCC.print_timings / Solver.print_timings
 *                                               lib/Preconditioner.py:252-260, lib/Solver.py:154-155
 *   pls_destroy         (object lifetime; PETSc XXXDestroy)
 *
 * Device-resident variants (inputs already in HBM, field-major order) exist
 * for benchmarks and for the synthetic generator of SURVEY.md 8(d).
 */
#ifndef PLS_H
#define PLS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PLS_ABI_VERSION 1

/* Host CSR (local rows): row_ptr[nrows+1] int64, col[nnz] int32, val[nnz] f64.
 * Columns inside a row must be sorted ascending (PETSc AIJ convention).       */
typedef struct pls_csr {
    int64_t nrows;
    int64_t ncols;
    const int64_t *row_ptr;
    const int32_t *col;
    const double *val;
} pls_csr;

typedef struct pls_handle pls_handle;
typedef struct pls_comm pls_comm;

/* Host allgather callback: every rank passes `bytes` bytes, receives
 * size * bytes (rank order) into recv.  Returns 0 on success.               */
typedef int (*pls_allgather_fn)(const void *send, int64_t bytes, void *recv, void *user);

/* Result of the last solve (KSPGetIterationNumber / KSPGetConvergedReason /
 * residual history as KSPSetResidualHistory records it).                      */
typedef struct pls_result {
    int32_t its;          /* outer iterations                                   */
    int32_t reason;       /* KSPConvergedReason value (AAR: 2 rtol, 3 atol, -3 its) */
    double rnorm;         /* last residual norm the outer solver tested        */
    int32_t pc_applies;   /* block-PC applications during the solve            */
    int32_t history_len;  /* entries available through pls_get_history         */
} pls_result;

/* Accumulated timers in seconds (names of lib/Preconditioner.py:35-39 and
 * lib/Solver.py:62), measured with HIP events on the solver stream.         */
typedef struct pls_timings {
    double pc_total;      /* t_total  */
    double pc_solid;      /* t_solid  */
    double pc_fluid;      /* t_fluid  */
    double pc_press;      /* t_press  */
    double pc_alloc;      /* t_alloc (field gathers/scatters; 0 in field-major layout) */
    double solver_total;  /* Solver.t_total */
    double spmv_total;    /* outer MatMult time */
    int64_t spmv_calls;
} pls_timings;

/* Synthetic 3-field system; generated directly in HBM.     */
typedef struct pls_synth_spec {
    int32_t dim;          /* 2 or 3                                            */
    int32_t N;            /* elements per side                                 */
    uint64_t seed;
    double delta;         /* diagonal shift                                    */
} pls_synth_spec;

int pls_abi_version(void);
const char *pls_last_error(void);
int pls_device_count(int *count);
int pls_set_device(int device);

/* Options: newline-separated "key value" (or "key") lines.  Keys prefixed
 * "pls." are the reference's parameter dict entries ("pls.solver_type gmres",
 * "pls.pc_type diagonal", "pls.inner_ksp_type preonly", ...); every other key
 * is a PETSc options-database entry without its leading '-' ("s_pc_type ilu",
 * "global_ksp_pc_side right", ...), resolved with setFromOptions precedence. */

/* Build a solver from host CSR matrices in the caller's (e.g. dolfin
 * interleaved) ordering plus the field index sets (sorted global indices of
 * each field, lib/IndexSet.py:38-41).  Pdiff may be NULL unless pc type is a
 * 3-way variant.  bcs_sub_p: positions inside the p sub-vector with pressure
 * Dirichlet BCs (lib/Poromechanics.py:48-55).                               */
int pls_create(const pls_csr *A, const pls_csr *P, const pls_csr *Pdiff,
               const int32_t *is_s, int64_t ns, const int32_t *is_f, int64_t nf,
               const int32_t *is_p, int64_t np, const int32_t *bcs_sub_p, int64_t nbc,
               const char *options, pls_handle **out);

/* Build a solver whose A, P, P_diff, index sets and pressure BCs come from the
 * seeded synthetic generator, directly on the device, field-major order.     */
int pls_create_synthetic(const pls_synth_spec *spec, const char *options, pls_handle **out);

/* ---- distributed solve (one process per GPU) ----------
 * Row slabs per field (PETSc ownership split), halo exchange before each
 * SpMV, deterministic global sums (allgather + rank-ordered sum), block-Jacobi
 * inner blocks per rank.  Replaces the reference's MPI data parallelism
 * (mpirun -np 8, paper-scripts/robustness_2d.sh:29; PETSc MPIAIJ + VecScatter,
 * lib/Solver.py:151, lib/Preconditioner.py:170-234).                        */
int pls_rccl_unique_id(char out[128]);
int pls_comm_create_rccl(const char id[128], int rank, int size, pls_comm **out);
int pls_comm_create_callback(int rank, int size, pls_allgather_fn fn, void *user, pls_comm **out);
int pls_comm_destroy(pls_comm *comm);
/* Each rank generates and owns its slabs of the synthetic system; the handle
 * must be destroyed before its communicator.  Vectors of the device entry
 * points are rank-local ([s_r | f_r | p_r]).                                 */
int pls_create_synthetic_dist(const pls_synth_spec *spec, const char *options, pls_comm *comm, pls_handle **out);
/* Mean latency of one global sum of `count` doubles (allgather + rank-ordered
 * sum + the stream sync the Krylov loop performs), over `reps` calls; the
 * reference's MPI_Allreduce inside VecMDot / VecNorm.                       */
int pls_bench_global_sum(pls_handle *h, int32_t count, int32_t reps, double *sec_per_call);
/* Multi-rank pls_create from the caller's matrices -- what the reference
 * drivers hold under mpirun (paper-scripts/robustness_2d.sh:29): on every rank
 * A, P, P_diff are the rank's MPIAIJ rows (A.getValuesCSR() of the operator of
 * lib/Solver.py:151: nrows = this rank's rows, ncols = the global n, global
 * column indices), rows [row_start, row_start + ns + nf + np) of the global
 * (dolfin) numbering; is_s / is_f / is_p are the global indices of the dofs
 * this rank owns (dofmap().dofs(), lib/IndexSet.py:38-41; 2-way: fp = their
 * sorted union, the all-gather of lib/IndexSet.py:49 happens inside);
 * bcs_sub_p = positions inside this rank's p sub-vector
 * (lib/Poromechanics.py:48-55).  Field blocks take the row ownership of the
 * rank-local index sets, as PETSc's createSubMatrix (lib/Preconditioner.py:
 * 61-74) gives them.  Collective over comm; host vectors of pls_solve /
 * pls_pc_apply / pls_matmult are this rank's rows in the caller's order.   */
int pls_create_dist(const pls_csr *A, const pls_csr *P, const pls_csr *Pdiff, int64_t row_start, const int32_t *is_s,
                    int64_t ns, const int32_t *is_f, int64_t nf, const int32_t *is_p, int64_t np,
                    const int32_t *bcs_sub_p, int64_t nbc, const char *options, pls_comm *comm, pls_handle **out);

int pls_setup(pls_handle *h);
/* New values (or patterns) of A / P / P_diff (NULL: unchanged), caller's
 * ordering as in pls_create.  The block PC is set up again before the next
 * solve -- PETSc's PCSetUp on an operator state change, which the reference
 * triggers every time step by re-applying BCs to A and P
 * (lib/Poromechanics.py:70-86, lib/Solver.py:105 set_up).  Outer solver,
 * AAR and inner Anderson histories persist, as the reference's objects do. */
int pls_update_matrices(pls_handle *h, const pls_csr *A, const pls_csr *P, const pls_csr *P_diff);
/* Set / override one option ("key", "value" or NULL for a flag).  Options of
 * the outer solver ("pls.solver_*", "pls.aar_*", "global_*") may change until
 * pls_create_solver (or the first solve); PC options until pls_setup.        */
int pls_set_option(pls_handle *h, const char *key, const char *value);
/* Solver.create_solver (lib/Solver.py:64-103): build the outer KSP / AAR.    */
int pls_create_solver(pls_handle *h);
int pls_destroy(pls_handle *h);

/* Global size n and field sizes of a handle.                                 */
int pls_get_sizes(pls_handle *h, int64_t *n, int64_t *ns, int64_t *nf, int64_t *np, int64_t *nnz_A);

/* Host-vector entry points (caller's ordering, length n).                     */
int pls_pc_apply(pls_handle *h, const double *x, double *y);
int pls_solve(pls_handle *h, const double *b, double *x, pls_result *res);
int pls_matmult(pls_handle *h, const double *x, double *y);

/* Device-vector entry points: d_b / d_x are device pointers in the handle's
 * internal field-major order (no host traffic, no permutation).             */
int pls_solve_device(pls_handle *h, const double *d_b, double *d_x, pls_result *res);
int pls_pc_apply_device(pls_handle *h, const double *d_x, double *d_y);
int pls_matmult_device(pls_handle *h, const double *d_x, double *d_y);
/* Synthetic right-hand side (field-major) written to a device vector.        */
int pls_synthetic_rhs_device(pls_handle *h, uint64_t seed, double *d_b);
/* Device buffer helpers (so hosts without a GPU runtime binding can drive it) */
int pls_device_alloc(int64_t bytes, void **d_ptr);
int pls_device_free(void *d_ptr);
int pls_memcpy_h2d(void *d_dst, const void *h_src, int64_t bytes);
int pls_memcpy_d2h(void *h_dst, const void *d_src, int64_t bytes);

int pls_get_result(pls_handle *h, pls_result *res);
int pls_get_history(pls_handle *h, double *hist, int32_t cap);
int pls_get_timings(pls_handle *h, pls_timings *t);
int pls_reset_timings(pls_handle *h);
/* Totals of one inner (or the outer) KSP since the handle's setup, by options
 * prefix ("s_", "f_", "p_", "diff_", "fp_", "fp_fieldsplit_0_", ..., "global_"):
 * stats[0] solves, [1] iterations, [2] most iterations of one solve, [3] solves
 * that ended with a negative KSPConvergedReason (PETSc's -ksp_converged_reason
 * per solve, summed; the reference's own output is the outer count only,
 * lib/AbstractPhysics.py:77-78), [4] the most recent such reason (0: none).  */
int pls_get_ksp_stats(pls_handle *h, const char *prefix, int64_t stats[5]);

/* Export a device matrix of the handle to host CSR (tests / parity):
 * which: 0 = A, 1 = P, 2 = P_diff (field-major order).  Call once with
 * col == NULL to get nrows/nnz, then with buffers sized accordingly.        */
int pls_export_matrix(pls_handle *h, int which, int64_t *nrows, int64_t *nnz,
                      int64_t *row_ptr, int32_t *col, double *val);
/* Export the field-major permutation: perm[internal] = caller index.         */
int pls_get_permutation(pls_handle *h, int64_t *perm);

/* Host-only query of the classical AMG behind -pc_type hypre (no device
 * needed; test and inspection entry): level `level` of the hierarchy that
 * options' <prefix>pc_hypre_boomeramg_* build from A (petsc-options-inexact:
 * 16-24): n, nc, nnz of P (of the coarsest operator when level ==
 * *nlevels - 1); when non-NULL, cf[n] (1 C / -1 F) and P's CSR arrays
 * (p_rp[n + 1], p_ci[nnz], p_v[nnz]).                                        */
int pls_boomeramg_host_level(const pls_csr *A, const char *options, const char *prefix, int64_t level,
                             int64_t *nlevels, int64_t *n, int64_t *nc, int64_t *p_nnz, int8_t *cf, int64_t *p_rp,
                             int32_t *p_ci, double *p_v);

/* Host-only analysis of the sparse LU (the MUMPS stand-in behind -pc_type lu
 * past pls.lu_dense_max rows; petsc-options-exact:11-35,
 * petsc-options-inexact:105-106) that `options` would build on A: ordering
 * (pls.lu_nd*) and symbolic factorization only, no device needed.
 * stats[0..9]: n, fronts, tree levels, largest front (p + q), factor doubles
 * stored and read once per solve (sum p (p + 2 q)), the fronts' dense
 * workspace doubles (64-row tiles, summed over fronts), factorization flops,
 * ordering s, symbolic s, largest separator.  When non-NULL: perm[n] (ND
 * position -> row), front_of[n] (position -> front, fronts numbered in
 * postorder so every front's pivots are contiguous) and parent[fronts]
 * (-1 at the root); call with them NULL first to learn the front count.    */
int pls_sparse_lu_analyze(const pls_csr *A, const char *options, double *stats, int64_t nstats, int32_t *perm,
                          int32_t *front_of, int32_t *parent);

/* Standalone inner Anderson mixing (lib/AndersonAcceleration.py:8-78): the
 * object a caller's own fixed-point loop holds, as the reference's
 * PreconditionerCC holds one per inner block (lib/Preconditioner.py:248-249).
 *   pls_anderson_create   AndersonAcceleration(order), vectors of length n
 *                         (AndersonAcceleration.py:8-17)
 *   pls_anderson_next     get_next_vector(gk) (AndersonAcceleration.py:19-78):
 *                         d_gk (device, length n) is replaced by the mixed
 *                         iterate x_k, in place as the reference's
 *                         self.xk.copy(gk); F / X histories persist across
 *                         calls, the least squares is Householder QR (TSQR)
 *   pls_anderson_destroy  frees the object and its stream.
 * Single-rank: the reference's scatter-to-rank-0 least squares over MPI is
 * the handle's inner accel path (option pls.inner_accel_order) at G > 1.    */
typedef struct pls_anderson pls_anderson;
int pls_anderson_create(int32_t order, int64_t n, pls_anderson **out);
int pls_anderson_next(pls_anderson *a, double *d_gk);
int pls_anderson_destroy(pls_anderson *a);

/* Kernel micro-entry points used by bench.py's roofline leg (device ptrs):
 * y = A x on the handle's A, repeated `reps` times; returns the mean device
 * time per launch in seconds measured with HIP events on the solver stream. */
int pls_bench_spmv(pls_handle *h, const double *d_x, double *d_y, int32_t reps, double *sec_per_launch);
/* Layout of A's SpMV copy: d16 = 1 for SELL-64/D16 (16-bit column deltas),
 * 0 for SELL-64 (int32 columns); matrix_bytes = bytes one product streams
 * from the matrix arrays (padding included).  Option "pls.sell_d16 0"
 * forces the int32 layout.                                                   */
int pls_spmv_layout(pls_handle *h, int32_t *d16, int64_t *matrix_bytes);
/* Streaming probe on the current device: per repetition `bytes` read (and,
 * unless read_only, `bytes` written) with 16-B-per-lane nontemporal accesses;
 * returns GB/s of bytes moved -- the achievable HBM rate beside the 8 TB/s
 * peak.                                                     */
int pls_bench_copy(int64_t bytes, int32_t reps, int32_t read_only, double *gbs);

#ifdef __cplusplus
}
#endif
#endif /* PLS_H */
