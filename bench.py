"""Benchmark: Krylov iterations/s of the block-preconditioned GMRES hot path on MI355X.

Workload (BASELINE.json metric "Krylov iters/sec + SpMV achieved HBM GB/s,
3-field poroelastic 10M DoF"): the synthetic 3-field system of SURVEY.md 8(d)
at 3-D N=59 (10,326,954 DoF, ~1.88 G nnz in A), generated in HBM; one step =
one full outer solve from a zero guess exactly as the reference runs it
(``Solver.solve``: right-preconditioned GMRES, rtol 1e-6, atol 1e-8, restart =
maxit = 100, swelling-3d.py:64-66) with the 2-way block preconditioner
(lib/Preconditioner.py:219-246) and inner PREONLY + BJACOBI(ILU(0)) blocks.

value = whole-job Krylov iterations per second on the 10.33M-DoF system.  At
G GPUs the solve is sharded the way the reference runs under MPI (one process
per GPU, PETSc row slabs of every field, halo exchange before each SpMV,
rank-ordered global sums, BJACOBI blocks inside each rank; RCCL over xGMI, see
DESIGN.md §6).  ``--scaling strong`` (the default at G > 1; north_star's
"RCCL-dot scaling"): the same N=59 system on G GPUs with the same TOTAL
BJACOBI block counts (PETSc's -pc_bjacobi_blocks is a total), value = outer
iterations / max-over-ranks time.  ``--scaling weak``: a global system G
times as large (3-D N = round(59 G^(1/3)), ~10.3M DoF and 256/264 blocks per
GPU); one outer iteration there is worth n_global / 10,326,954 iterations of
the metric's system.  ``--scaling replicas``: G independent N=59 solves.

roofline: the dominant kernel is the CSR SpMV with A (one per outer
iteration).  achieved = algorithmic bytes per launch
(12 nnz + 8 (n+1) + 8 n + 8 n: val + col + int64 row_ptr + x once + y once)
divided by the mean SpMV duration measured with HIP events on the solver
stream inside the timed solves; peak = 8000 GB/s (MI355X HBM3E).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "poroelasticity-linear-solvers_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "Krylov iters/sec + SpMV achieved HBM GB/s, 3-field poroelastic 10M DoF"
HBM_PEAK_GBS = 8000.0
SEED = 20261015
DELTA = 0.05
RHS_SEED = 7  # the seed of the device-generated right-hand side (pls_synthetic_rhs_device)


# reference petsc-options-inexact (BoomerAMG -> the device classical AMG,
# MUMPS -> the device LU): CG on s/f/p, PREONLY on diff, Schur fieldsplit on fp
INEXACT_DB = {
    "global_ksp_type": "gmres", "global_ksp_norm_type": "unpreconditioned",
    "s_ksp_type": "cg", "s_ksp_norm_type": "unpreconditioned", "s_ksp_atol": "0.0", "s_ksp_rtol": "1e-1",
    "s_pc_type": "hypre", "s_pc_hypre_boomeramg_grid_sweeps_all": "1",
    "f_ksp_type": "cg", "f_ksp_norm_type": "unpreconditioned", "f_ksp_atol": "0.0", "f_ksp_rtol": "1e-2",
    "f_pc_type": "hypre", "f_pc_hypre_boomeramg_grid_sweeps_all": "1",
    "p_ksp_type": "cg", "p_ksp_norm_type": "unpreconditioned", "p_ksp_atol": "0.0", "p_ksp_rtol": "1e-2",
    "p_pc_type": "hypre", "diff_ksp_type": "preonly", "diff_pc_type": "hypre",
    "fp_ksp_type": "preonly", "fp_pc_fieldsplit_type": "schur", "fp_pc_fieldsplit_schur_fact_type": "lower",
    "fp_pc_fieldsplit_schur_precondition": "selfp",
    "fp_fieldsplit_0_ksp_type": "cg", "fp_fieldsplit_0_ksp_rtol": "1e-4", "fp_fieldsplit_0_ksp_atol": "0.0",
    "fp_fieldsplit_0_ksp_max_it": "10", "fp_fieldsplit_0_pc_type": "hypre",
    "fp_fieldsplit_1_ksp_type": "preonly", "fp_fieldsplit_1_pc_type": "lu",
}
# petsc-options-inexact's BoomerAMG settings (:16-24 and the other blocks)
BOOMER = {"pc_hypre_boomeramg_P_max": "4", "pc_hypre_boomeramg_agg_nl": "1", "pc_hypre_boomeramg_agg_num_paths": "2",
          "pc_hypre_boomeramg_coarsen_type": "HMIS", "pc_hypre_boomeramg_interp_type": "ext+i",
          "pc_hypre_boomeramg_no_CF": "true"}
for _pre in ("s_", "f_", "p_", "diff_", "fp_fieldsplit_0_"):
    INEXACT_DB.update({_pre + k: v for k, v in BOOMER.items()})


# BASELINE.json "configs": named presets (dim, N, option set); the default is
# configs[1] at the metric's size.  Only the metric's configuration is the
# headline bench line; the others are measured and recorded in DESIGN.md.
CONFIGS = {
    # configs[0]: swelling.py 2-D N=32, exact block PC (petsc-options-exact:
    # right-PC GMRES, PREONLY + LU on every block; MUMPS -> device LU),
    # swelling.py:63-67 atol 1e-8 rtol 1e-6 maxit 500
    "swelling2d-exact": dict(dim=2, N=32, maxit=500, atol=1e-8, preset="exact", cpu_N=32),
    # configs[1] (metric: N=59 = 10.33M DoF; N=64 is the named size)
    "swelling3d-bjacobi": dict(dim=3, N=59, maxit=100, atol=1e-8, preset=None),
    # configs[2]: footing.py at N=128 (2-D in the reference: footing.py:18-19;
    # its local refinement near the footing is not modelled by the synthetic
    # system) with petsc-options-inexact and ILU(0) in place of BoomerAMG: CG
    # blocks, Schur lower/selfp fieldsplit on fp (Schur block: device LU).
    # footing.py:73-76 atol 1e-4 maxit 500.
    "footing-inexact-ilu": dict(dim=2, N=128, maxit=500, atol=1e-4, preset="inexact-ilu", cpu_N=48),
    # footing.py's own inner PC ("inner pc type" hypre, footing.py:73) with
    # petsc-options-inexact itself: BoomerAMG -> the classical AMG
    "footing-inexact": dict(dim=2, N=128, maxit=500, atol=1e-4, preset=None, inexact=True, cpu_N=12),
    # configs[4]: AAR depth m=5 (sharded across ranks under torchrun)
    "aar-m5": dict(dim=3, N=59, maxit=100, atol=1e-8, preset=None, solver="aar", aar_order=5, cpu_N=20),
}


def _inexact_db(amg: str, blocks: int = 64):
    """petsc-options-inexact with BoomerAMG replaced by ILU(0) blocks: block
    Jacobi with ILU(0) sub-blocks (PETSc's parallel ILU; one workgroup per
    block in LDS on the device), ``blocks`` blocks per inner PC."""
    db = dict(INEXACT_DB)
    if amg == "ilu":
        for k in list(db):
            if db[k] == "hypre":
                pre = k[:-len("pc_type")]
                db[k] = "bjacobi"
                db[pre + "pc_bjacobi_blocks"] = str(blocks)
                db[pre + "sub_pc_type"] = "ilu"
            if "hypre" in k:
                del db[k]
    return db


def solver_options(args):
    three = args.pc_type == "diagonal 3-way"
    if args.preset == "exact":
        params = {"solver type": args.solver, "solver atol": args.atol, "solver rtol": 1e-6,
                  "solver maxiter": args.maxit, "pc type": args.pc_type, "inner ksp type": "preonly",
                  "inner pc type": "lu", "inner accel order": 0, "AAR order": args.aar_order, "AAR p": 5,
                  "AAR omega": 1.0, "AAR beta": 1.0}
        db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right"}
        for pre in (("s_", "f_", "p_", "diff_") if three else ("s_", "fp_")):
            db[pre + "ksp_type"] = "preonly"
            db[pre + "pc_type"] = "lu"
        return params, db
    if args.preset == "inexact-ilu":
        params = {"solver type": args.solver, "solver atol": args.atol, "solver rtol": 1e-6,
                  "solver maxiter": args.maxit, "pc type": args.pc_type, "inner ksp type": "cg",
                  "inner pc type": "ilu", "inner accel order": 0, "AAR order": args.aar_order, "AAR p": 5,
                  "AAR omega": 1.0, "AAR beta": 1.0}
        return params, _inexact_db("ilu", args.blocks_inner)
    if args.inexact:
        params = {"solver type": args.solver, "solver atol": args.atol, "solver rtol": 1e-6,
                  "solver maxiter": args.maxit, "pc type": args.pc_type, "inner ksp type": "cg",
                  "inner pc type": "hypre", "inner accel order": 0, "AAR order": args.aar_order, "AAR p": 5,
                  "AAR omega": 1.0, "AAR beta": 1.0}
        return params, dict(INEXACT_DB)
    params = {"solver type": args.solver, "solver atol": args.atol, "solver rtol": 1e-6, "solver maxiter": args.maxit,
              "pc type": args.pc_type, "inner ksp type": "preonly", "inner pc type": args.inner,
              "inner accel order": 0, "AAR order": args.aar_order, "AAR p": 5, "AAR omega": 1.0, "AAR beta": 1.0}
    db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right"}
    if args.inner in ("gamg", "hypre"):
        # AMG on the field blocks; the coupled 2-way fp block keeps BJACOBI(ILU(0))
        for pre in (("s_", "f_", "p_", "diff_") if three else ("s_",)):
            db[pre + "ksp_type"] = "preonly"
            db[pre + "pc_type"] = args.inner
            if args.inner == "hypre":
                db.update({pre + k: v for k, v in BOOMER.items()})
        if not three:
            db.update({"fp_ksp_type": "preonly", "fp_pc_type": "bjacobi", "fp_pc_bjacobi_blocks": str(args.blocks_fp)})
            params["inner pc type"] = "bjacobi"
        return params, db
    # block counts: every block solution fits one CU's LDS (<= 20480 rows)
    blocks = {"s_": args.blocks_s, "fp_": args.blocks_fp, "f_": args.blocks_s, "p_": args.blocks_p,
              "diff_": args.blocks_p}
    for pre in (("s_", "f_", "p_", "diff_") if three else ("s_", "fp_")):
        db[pre + "ksp_type"] = "preonly"
        db[pre + "pc_type"] = args.inner
        if args.inner == "bjacobi":
            db[pre + "pc_bjacobi_blocks"] = str(blocks[pre])
    return params, db


def cpu_baseline(args, params, db):
    """The same configuration on the host cores, timed on a bounded sample.

    bench's configuration (2-way, GMRES, PREONLY + BJACOBI(ILU(0))) runs the
    C/OpenMP restatement oracle/csrc/cpu_solver.c on all available cores
    (SURVEY.md 8(d)'s planned baseline) on the benched system itself (same
    matrices, same iteration count); other configurations fall back to the
    single-thread Python oracle on a smaller sample, iters/s scaled by DoF to
    the benched system (the per-iteration work is linear in n)."""
    from oracle import synthetic as S
    Ns = args.cpu_N
    if args.system == "fe":
        return _cpu_baseline_fe(args, params, db)
    spec = S.SynthSpec(args.dim, Ns, SEED, DELTA)
    t0 = time.perf_counter()
    A, P = S.matrix(spec, 0), S.matrix(spec, 1)
    # the right-hand side the device solves (h.rhs_device(7, ...): seed 7)
    b = S.rhs(S.SynthSpec(args.dim, Ns, RHS_SEED, DELTA))
    n_sample = spec.n
    n_metric = S.SynthSpec(args.dim, args.N).n if args.N != Ns else n_sample
    c_path = (params["pc type"] == "diagonal" and params["solver type"] == "gmres" and args.inner == "bjacobi"
              and not args.inexact and args.preset is None)
    if c_path:
        from oracle import native
        try:
            cores = len(os.sched_getaffinity(0))
        except AttributeError:
            cores = os.cpu_count() or 1
        cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores) or cores))
        t_gen = time.perf_counter() - t0
        _, its, reason, _, t_setup, dt = native.cpu_gmres_2way(
            A, P, spec.sizes()[0], args.blocks_s, args.blocks_fp, b, rtol=params["solver rtol"],
            atol=params["solver atol"], maxit=args.cpu_maxit, nthreads=cores)
        rate = its / dt
        same = n_sample == n_metric
        return {"value": rate * n_sample / n_metric,
                "unit": f"Krylov iters/s (scaled by DoF to the {n_metric}-DoF system)", "cores": cores, "kind": "port",
                "sample": (f"oracle/csrc/cpu_solver.c (C + OpenMP, {cores} threads): bench's configuration on "
                           f"the N={Ns} {args.dim}-D system ({n_sample} DoF, {A.nnz} nnz), {its} GMRES iterations in "
                           f"{dt:.1f}s (block setup {t_setup:.1f}s, generation {t_gen:.1f}s), reason {reason}"
                           + ("; the benched system itself, no scaling" if same else
                              f"; iters/s x {n_sample}/{n_metric}")),
                "raw_iters_per_s": rate, "its": its, "petsc4py": _petsc_probe()}
    from oracle.solver import OracleSolver
    three = params["pc type"] == "diagonal 3-way"
    Pd = S.matrix(spec, 2) if three else None
    is_s, is_f, is_p = S.field_major_index_sets(spec)
    p = dict(params)
    p["solver maxiter"] = args.cpu_maxit
    o = OracleSolver(A, P, Pd, is_s, is_f, is_p, p, db, S.bcs_sub_pressure(spec) if three else [])
    t_setup = time.perf_counter() - t0
    t1 = time.perf_counter()
    o.solve(b)
    dt = time.perf_counter() - t1
    rate = o.its / dt
    return {"value": rate * n_sample / n_metric, "unit": f"Krylov iters/s (scaled by DoF to the {n_metric}-DoF system)",
            "cores": 1, "kind": "port",
            "sample": (f"oracle (numpy/scipy + C kernels, 1 thread) {params['pc type']} / {params['solver type']} "
                       f"solve of the N={Ns} {args.dim}-D system ({n_sample} DoF), {o.its} outer iterations in {dt:.1f}s "
                       f"(setup {t_setup:.1f}s), maxit {args.cpu_maxit}; iters/s x {n_sample}/{n_metric}"),
            "raw_iters_per_s": rate}


def _petsc_probe():
    """time the reference's own PETSc path if petsc4py is already
    installed on the box (never installed here).  Records the outcome."""
    try:
        import importlib.util
        spec = importlib.util.find_spec("petsc4py")
    except (ImportError, ValueError):
        spec = None
    return "present (not timed: the reference's dolfin assembly is absent)" if spec else "absent on this host"


def _cpu_baseline_fe(args, params, db):
    """--system fe: the Python oracle (1 thread) on the assembled swelling
    system at N = cpu_N, iters/s scaled by DoF to the benched system."""
    from lib.fe_swelling import assemble_swelling
    from lib.fe_footing import assemble_footing, footing_dofs
    from oracle.solver import OracleSolver
    t0 = time.perf_counter()
    footing = args.config.startswith("footing")
    if footing:
        fe = assemble_footing(args.cpu_N, params["pc type"])
    else:
        fe = assemble_swelling(args.dim, args.cpu_N, params["pc type"])
    n_sample = fe.A.shape[0]
    n_metric = n_sample if args.N == args.cpu_N else footing_dofs(args.N) if footing else (
        6 * (2 * args.N + 1) ** 3 + (args.N + 1) ** 3 if args.dim == 3 else 4 * (2 * args.N + 1) ** 2 + (args.N + 1) ** 2)
    p = dict(params)
    p["solver maxiter"] = args.cpu_maxit
    o = OracleSolver(fe.A, fe.P, fe.P_diff, fe.is_s, fe.is_f, fe.is_p, p, db, fe.bcs_sub_pressure)
    o.solve(fe.b)  # first solve sets the inner PCs up (lazily, as PETSc does); time the second
    t_setup = time.perf_counter() - t0
    t1 = time.perf_counter()
    o.solve(fe.b)
    dt = time.perf_counter() - t1
    rate = o.its / dt
    return {"value": rate * n_sample / n_metric, "unit": f"Krylov iters/s (scaled by DoF to the {n_metric}-DoF system)",
            "cores": 1, "kind": "port",
            "sample": (f"oracle (numpy/scipy + C kernels, 1 thread) {params['pc type']} / {params['solver type']} "
                       f"solve of the assembled N={args.cpu_N} {args.dim}-D swelling system ({n_sample} DoF), {o.its} "
                       f"outer iterations in {dt:.2f}s (second solve; assembly + setup + first solve {t_setup:.1f}s); iters/s x {n_sample}/{n_metric}")
                       .replace("swelling system", "footing system" if footing else "swelling system"),
            "raw_iters_per_s": rate}


def shard_plan(args, world):
    """(sharded, global N) for G = world ranks; weak scaling also scales the
    total BJACOBI block counts (blocks per GPU fixed), strong scaling keeps the
    single-GPU system and its total block counts (PETSc's -pc_bjacobi_blocks
    is a total over the ranks)."""
    if args.replicas:
        args.scaling = "replicas"
    sharded = world > 1 and args.scaling != "replicas"
    N_glob = args.N
    if sharded and args.scaling == "weak":
        N_glob = int(round(args.N * world ** (1.0 / args.dim)))
        args.blocks_s *= world
        args.blocks_fp *= world
        args.blocks_p *= world
    return sharded, N_glob


def launch_plan(gpus, env):
    """How this process runs ``--gpus G`` (the reference's ``mpirun -np G``,
    paper-scripts/robustness_2d.sh:29):

    * ``("run", G)``: this process is a rank of a G-rank job (WORLD_SIZE = G is
      set by torch.distributed.run) or G is 1;
    * ``("spawn", G)``: WORLD_SIZE is unset and G > 1 -- the caller must start G
      fresh rank processes (before any HIP call in this one) and exit with
      their status;
    * ``("error", msg)``: WORLD_SIZE disagrees with --gpus (a G-GPU line would
      otherwise report the wrong rank count).

    ``gpus`` None means "whatever WORLD_SIZE says" (1 outside a job)."""
    ws = env.get("WORLD_SIZE")
    if ws is None or ws == "":
        G = 1 if gpus is None else int(gpus)
        if G < 1:
            return "error", f"--gpus {G}: need at least one GPU"
        return ("spawn", G) if G > 1 else ("run", 1)
    W = int(ws)
    if gpus is not None and int(gpus) != W:
        return "error", f"--gpus {gpus} but WORLD_SIZE={W}: launch {gpus} ranks or pass --gpus {W}"
    return "run", W


def hypre_semantics(opts, ranks):
    """Which BoomerAMG run the classical AMG behind -pc_type hypre restates
    (oracle/boomeramg.py; csrc/boomeramg.cpp) under these options."""
    chunks = int(opts.get("pls.hypre_relax_chunks", 256))
    cch = int(opts.get("pls.hypre_coarsen_chunks", 1))
    crows = int(opts.get("pls.hypre_coarsen_min_rows", 65536))
    if opts.get("pls.hypre_ranks"):
        np_ = f"np = {opts['pls.hypre_ranks']} (pls.hypre_ranks)"
    elif ranks > 1 and opts.get("pls.hypre_dist", "1") not in ("0", "false"):
        np_ = f"np = {ranks} (the sharded block's ranks)"
    elif cch == 1:
        np_ = "np = 1"
    elif cch > 1:
        np_ = f"np = {cch} equal row partitions per level"
    else:
        np_ = (f"np = the most partitions <= min({chunks}, rows / {crows}) per level, halving until the "
               "partition boundaries cut <= 2 % of the strong connections (1 if none)")
    return {"coarsening": "HMIS = Ruge-Stueben first pass per process + PMIS stage (hypre_Rand measures, "
                          "seeds 2747 + process)", "processes": np_,
            "relax": (f"hybrid symmetric Gauss-Seidel (relax type 6) in K = {chunks} chunks per level "
                      f"(hypre's OpenMP threads), at least {int(opts.get('pls.hypre_relax_min_rows', 1024))} "
                      "rows per chunk"),
            "hypre_K": chunks, "relax_min_rows": int(opts.get("pls.hypre_relax_min_rows", 1024))}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(G, argv):
    """Run this script as a G-rank torch.distributed job (one process per GPU,
    LOCAL_RANK = GPU index) and return its exit status.  The parent imports
    nothing that touches the GPU; the ranks are fresh child processes (no exec
    of a process with an initialised GPU)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={G}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    print(f"[bench] --gpus {G}: launching {G} ranks (torch.distributed.run)", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def _progress(rank, msg):
    """Progress on stderr (rank 0): long configurations stay visibly alive;
    stdout carries only the JSON line."""
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="swelling3d-bjacobi", choices=sorted(CONFIGS),
                    help="BASELINE.json configuration preset (explicit flags override its fields)")
    ap.add_argument("--dim", type=int, default=3, choices=[2, 3])
    ap.add_argument("--atol", type=float, default=1e-8)
    ap.add_argument("--aar-order", type=int, default=10)
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment, G > 1 launches G ranks itself")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--N", type=int, default=59)
    ap.add_argument("--inner", default="bjacobi", choices=["bjacobi", "ilu", "jacobi", "gamg", "hypre"])
    ap.add_argument("--inexact", action="store_true",
                    help="the reference's petsc-options-inexact set (CG + AMG blocks, Schur fieldsplit on fp)")
    # block counts: one block per CU (256) for the solid block; 264 for the fp
    # block so every block solution (<= 20480 doubles = 160 KiB) fits one CU's LDS
    ap.add_argument("--blocks-s", type=int, default=256)
    ap.add_argument("--blocks-fp", type=int, default=264)
    ap.add_argument("--blocks-p", type=int, default=11, help="3-way p_ / diff_ blocks")
    ap.add_argument("--blocks-inner", type=int, default=64, help="footing preset: bjacobi blocks per inner PC")
    ap.add_argument("--maxit", type=int, default=100)
    ap.add_argument("--pc-type", default=None, choices=["diagonal", "diagonal 3-way", "3-way", "undrained"],
                    help="block preconditioner (the metric: 2-way 'diagonal'; --system fe with the footing "
                         "config: footing.py's 'undrained')")
    ap.add_argument("--solver", default="gmres", choices=["gmres", "aar"])
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-copy-probe", action="store_true", help="skip the device-copy bandwidth probe")
    # default: the CPU baseline solves the benched system itself (N=59: ~20-30 s on the box's 16 cores)
    ap.add_argument("--cpu-N", type=int, default=None)
    ap.add_argument("--cpu-maxit", type=int, default=100)
    ap.add_argument("--sell-d16", type=int, default=1, help="1: SELL-64/D16 SpMV layout (16-bit column deltas)")
    ap.add_argument("--d16-unroll", type=int, default=0, help="D16 SpMV: 8-entry groups per lane in flight (tuning)")
    ap.add_argument("--opt", action="append", default=[], help="extra library option key=value (diagnostics)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak", "replicas"],
                    help="G > 1: strong (same system, same total block counts), weak (G x the DoF), replicas")
    ap.add_argument("--replicas", action="store_true", help="alias of --scaling replicas")
    ap.add_argument("--system", default="synthetic", choices=["synthetic", "fe"],
                    help="fe: the P2-P2-P1 FE system assembled on the host, one GPU -- swelling "
                         "(lib/fe_swelling.py), or with --config footing-inexact-ilu footing.py's locally refined "
                         "system (lib/fe_footing.py)")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                    help="host: host-staged gloo communicator (ranks may share a GPU; rehearsal only)")
    pre, _ = ap.parse_known_args()
    preset = dict(CONFIGS[pre.config])
    ap.set_defaults(preset=preset.pop("preset"), **preset)
    args = ap.parse_args()
    mode, val = launch_plan(args.gpus, os.environ)
    if mode == "error":
        print(f"[bench] error: {val}", file=sys.stderr, flush=True)
        raise SystemExit(2)
    if (val > 1 and args.inner == "ilu" and not (args.replicas or args.scaling == "replicas")
            and "pls.redundant_ilu=1" not in args.opt):
        # PETSc's ILU refuses an MPIAIJ block (the library throws at setup): say so before launching
        print("[bench] error: --inner ilu on a block sharded over several ranks is what PETSc refuses "
              "(use --inner bjacobi, or --opt pls.redundant_ilu=1 for the one-rank ILU applied redundantly)",
              file=sys.stderr, flush=True)
        raise SystemExit(2)
    if mode == "spawn":
        raise SystemExit(spawn_ranks(val, sys.argv[1:]))
    footing_fe = args.system == "fe" and args.config.startswith("footing")
    if args.pc_type is None:
        args.pc_type = "undrained" if footing_fe else "diagonal"  # footing.py:71
    if args.pc_type == "3-way":
        args.pc_type = "diagonal 3-way"
    if args.cpu_N is None:
        args.cpu_N = args.N
    if footing_fe and "--cpu-N" not in sys.argv:
        args.cpu_N = 12  # the oracle's inner CG + BJACOBI(ILU) on the refined footing system: ~1 min at N=12

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # bootstrap + timing reductions; the solve talks RCCL

    import lib._native as Nat
    from lib.handle import Handle, params_to_options
    Nat.check(Nat.lib().pls_set_device(local if args.comm == "rccl" else 0))

    if args.system == "fe" and world > 1:
        raise SystemExit("--system fe runs on one GPU (the assembler is a host-side input generator)")
    sharded, N_glob = shard_plan(args, world)
    params, db = solver_options(args)
    opts = dict(db)
    opts.update(params_to_options(params))
    opts["pls.sell_d16"] = str(args.sell_d16)
    for kv in args.opt:
        k, _, v = kv.partition("=")
        opts[k] = v
    if args.d16_unroll:
        opts["pls.d16_unroll"] = str(args.d16_unroll)
    t0 = time.perf_counter()
    comm = None
    fe = None
    t_assembly = None
    if sharded:
        from lib.dist import Communicator
        comm = Communicator.rccl() if args.comm == "rccl" else Communicator.gloo()
        h = Handle.synthetic_dist(args.dim, N_glob, SEED, DELTA, opts, comm)
    elif args.system == "fe":
        if footing_fe:
            from lib.fe_footing import assemble_footing
            fe = assemble_footing(args.N, args.pc_type)
        else:
            from lib.fe_swelling import assemble_swelling
            fe = assemble_swelling(args.dim, args.N, args.pc_type)
        t_assembly = time.perf_counter() - t0
        _progress(rank, f"assembled the {args.dim}-D N={args.N} {'footing' if footing_fe else 'swelling'} system "
                        f"in {t_assembly:.1f} s")
        t0 = time.perf_counter()  # (setup_s: the library's, from the CSR hand-over; the assembly is the input generator)
        h = Handle.from_csr(fe.A, fe.P, fe.P_diff, fe.is_s, fe.is_f, fe.is_p, fe.bcs_sub_pressure, opts)
    else:
        h = Handle.synthetic(args.dim, args.N, SEED + rank, DELTA, opts)
    h.setup()
    h.create_solver()
    t_setup = time.perf_counter() - t0
    n, nnz = h.n, h.nnz_A
    _progress(rank, f"setup {t_setup:.2f} s ({n} DoF on this rank, nnz(A) {nnz})")
    d_b = Nat.DeviceArray(n)
    d_x = Nat.DeviceArray(n)

    def load_rhs():
        if fe is not None:
            d_b.upload(fe.b)
        else:
            h.rhs_device(RHS_SEED, d_b.p)
    load_rhs()

    for _ in range(args.warmup):
        tw = time.perf_counter()
        r = h.solve_device(d_b.p, d_x.p)
        _progress(rank, f"warmup solve: {r.its} its, reason {r.reason}, {time.perf_counter() - tw:.3f} s")
    h.reset_timings()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    t1 = time.perf_counter()
    its = 0
    reasons = []
    for _ in range(args.steps):
        r = h.solve_device(d_b.p, d_x.p)
        its += r.its
        reasons.append(r.reason)
    dt = time.perf_counter() - t1
    barrier()
    tm = h.timings()
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        it_t = torch.tensor([float(its)], dtype=torch.float64)
        dist.all_reduce(it_t, op=dist.ReduceOp.SUM)
        its_all = float(it_t.item())
    else:
        its_all = float(its)
    n_metric = 10326954  # DoF of the N=59 system the metric is quoted on
    n_global = n
    if sharded:
        import torch
        nt = torch.tensor([float(n)], dtype=torch.float64)
        dist.all_reduce(nt, op=dist.ReduceOp.SUM)
        n_global = int(nt.item())
        its_all = float(its) * n_global / n_metric  # every rank did the same its
    elif world == 1:
        n_metric = n

    spmv_avg = tm["spmv_total"] / max(1, tm["spmv_calls"])
    alg_bytes = 12.0 * nnz + 8.0 * (n + 1) + 8.0 * n + 8.0 * n
    achieved = alg_bytes / spmv_avg / 1e9 if spmv_avg > 0 else 0.0
    iso = h.bench_spmv(d_x.p, d_b.p, 10)
    # latency of the solve's global sums: a CGS step's k+1 dots (k ~ its/2) and a norm
    # (sharded runs only: a single rank's "global" sum is a local reduction)
    gsum_us = ({"dots_40": 1e6 * h.bench_global_sum(40, 50), "norm_1": 1e6 * h.bench_global_sum(1, 50)}
               if sharded else None)
    d16, mat_bytes = h.spmv_layout()
    fmt_bytes = mat_bytes + 8.0 * n + 8.0 * n  # + x once + y once
    load_rhs()

    # achievable streaming bandwidth on this box: a 4 GiB
    # device-to-device copy (pls_bench_copy), read + write bytes / time
    copy_gbs = None
    if rank == 0 and not args.no_copy_probe:
        import ctypes as C
        g, gr = C.c_double(), C.c_double()
        Nat.check(Nat.lib().pls_bench_copy(1 << 32, 10, 0, C.byref(g)))
        Nat.check(Nat.lib().pls_bench_copy(1 << 32, 10, 1, C.byref(gr)))
        copy_gbs = {"copy": g.value, "read": gr.value}

    # HBM traffic of the same kernel from the committed PMC passes (tools/pmc.sh)
    traffic, traffic_src = None, None
    kname = ("void pls::k_d16_spmv<4, 1, false" if d16 else "void pls::k_sell_spmv<8, 1, false")  # any unroll
    pmc = next((q for q in (os.path.join(ROOT, "profiles", f"r{r:02d}_pmc_N59_summary.json") for r in range(9, 0, -1))
                if os.path.exists(q)), "")  # the latest round's committed PMC passes
    if os.path.exists(pmc) and n_global == 10326954 and world == 1 and fe is None:
        for k, v in json.load(open(pmc)).items():
            if k.startswith(kname) and v.get("read_bytes"):
                traffic = v["read_bytes"] + (v.get("write_bytes") or 0.0)
                traffic_src = os.path.relpath(pmc, ROOT)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": its_all / dt,
            "unit": ("Krylov iters/s (outer GMRES iterations on the 10.33M-DoF system; sharded runs: "
                     "iterations x n_global/10.33M)"),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * dt / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if (world == 1 or args.scaling == "strong") else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (seeded SPD 3-field block system, SURVEY.md 8(d); generated in HBM)" if fe is None else
                     "P2-P2-P1 footing FE system (lib/fe_footing.py: footing.py's twice locally refined mesh, "
                     "traction and BCs; lib/Assembler.py's forms, first time step; assembled on the host, copied to "
                     "HBM before timing)" if footing_fe else
                     "P2-P2-P1 swelling FE system (lib/fe_swelling.py: lib/Assembler.py's forms, first time step; "
                     "assembled on the host, copied to HBM before timing)"),
            "config": {
                "workload": (f"{args.config}"
                             f"{(' on the assembled ' + ('footing' if footing_fe else 'swelling') + ' FE system') if fe is not None else ''}: "
                             f"{args.dim}-D N={N_glob} ({n_global} DoF): outer "
                             + ("GMRES right-PC" if args.solver == "gmres" else f"AAR({args.aar_order}, p=5)")
                             + f" rtol 1e-6 atol {args.atol:g} maxit={args.maxit}, "
                             + ("3-way" if "3-way" in args.pc_type else "2-way") + f" '{args.pc_type}' block PC, "
                             + ("petsc-options-exact (PREONLY + LU blocks)" if args.preset == "exact" else
                                "petsc-options-inexact with ILU(0) for BoomerAMG (CG blocks, Schur fieldsplit fp)"
                                if args.preset == "inexact-ilu" else
                                "petsc-options-inexact (CG + AMG blocks, Schur fieldsplit fp)" if args.inexact else
                                "inner preonly+" + args.inner
                                + (f"(ILU(0), {args.blocks_s}/{args.blocks_fp} blocks s/fp)"
                                   if args.inner == "bjacobi" else ""))),
                "dim": args.dim, "N": N_glob, "dofs": n_global, "dofs_rank0": n, "nnz_A_rank0": nnz,
                "parallelism": (f"row slabs x{world} ({args.comm}, {args.scaling} scaling)" if sharded else
                                f"replicas x{world}" if world > 1 else "single GPU"),
            },
            "its_per_solve": its / args.steps,
            "comm": ({"global_sum_latency_us": gsum_us, "spmv_gbs_rank0": achieved,
                      "note": "per-rank SpMV includes the halo exchange it waits for"} if sharded else
                     {"global_sum_latency_us": None, "note": "one rank per solve: no communication"}),
            "reasons": sorted(set(reasons)),
            "setup_s": t_setup,
            "assembly_s": t_assembly,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "stream_gbs_measured": copy_gbs,
                         "kernel": ("k_d16_spmv<4,1,false>" if d16 else "k_sell_spmv<8,1,false>") + " (y = A x, outer MatMult)",
                         "alg_bytes_per_launch": alg_bytes, "mean_launch_s": spmv_avg,
                         "isolated_spmv_gbs": alg_bytes / iso / 1e9,
                         "layout": "SELL-64/D16 (16-bit column deltas)" if d16 else "SELL-64 (int32 columns)",
                         "layout_bytes_per_launch": fmt_bytes,
                         "layout_gbs": fmt_bytes / spmv_avg / 1e9 if spmv_avg > 0 else 0.0},
            "timings_s": {k: v for k, v in tm.items()},
        }
        if any(v == "hypre" for k, v in opts.items() if k.endswith("pc_type")):
            out["hypre_semantics"] = hypre_semantics(opts, world if sharded else 1)
        if not args.no_cpu and world == 1:
            _progress(rank, f"cpu baseline on the N={args.cpu_N} sample ...")
            out["cpu_baseline"] = cpu_baseline(args, params, db)
        print(json.dumps(out))
    d_b.free()
    d_x.free()
    h.destroy()
    if comm is not None:
        comm.destroy()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
