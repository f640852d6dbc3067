"""bench.py's BASELINE.json presets (host logic, no GPU): each configuration
maps to the reference's option sets as DESIGN.md §5 states.

* swelling2d-exact: petsc-options-exact (right-PC GMRES, PREONLY + LU on every
  block; reference petsc-options-exact:3-35), swelling.py:63-67 tolerances;
* footing-inexact-ilu: petsc-options-inexact with every BoomerAMG block
  replaced by BJACOBI(ILU(0)) and the Schur block's MUMPS LU kept as LU
  (petsc-options-inexact:12-114), footing.py atol 1e-4;
* swelling3d-bjacobi: the headline (2-way, PREONLY + BJACOBI(ILU(0)) 256 / 264
  blocks), N = 59;
* aar-m5: AAR with depth 5 (BASELINE configs[4]).
"""
import argparse
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _args(config, **over):
    a = dict(bench.CONFIGS[config])
    preset = a.pop("preset")
    ns = argparse.Namespace(config=config, dim=3, atol=1e-8, aar_order=10, N=59, inner="bjacobi", inexact=False,
                            blocks_s=256, blocks_fp=264, blocks_p=11, blocks_inner=64, maxit=100,
                            pc_type="diagonal", solver="gmres", cpu_N=40, cpu_maxit=100, preset=preset)
    for k, v in a.items():
        setattr(ns, k, v)
    for k, v in over.items():
        setattr(ns, k, v)
    return ns


def test_every_preset_names_a_known_configuration():
    assert set(bench.CONFIGS) == {"swelling2d-exact", "swelling3d-bjacobi", "footing-inexact-ilu", "footing-inexact", "aar-m5"}
    assert bench.CONFIGS["swelling3d-bjacobi"]["N"] == 59  # the metric's 10.33M-DoF system


def test_exact_preset_is_preonly_lu_everywhere():
    params, db = bench.solver_options(_args("swelling2d-exact"))
    assert params["solver maxiter"] == 500 and params["solver atol"] == 1e-8
    assert db["global_ksp_pc_side"] == "right"
    for pre in ("s_", "fp_"):
        assert db[pre + "ksp_type"] == "preonly" and db[pre + "pc_type"] == "lu"
    _, db3 = bench.solver_options(_args("swelling2d-exact", pc_type="diagonal 3-way"))
    for pre in ("s_", "f_", "p_", "diff_"):
        assert db3[pre + "pc_type"] == "lu"


def test_footing_preset_replaces_boomeramg_by_ilu_blocks():
    params, db = bench.solver_options(_args("footing-inexact-ilu"))
    assert params["solver atol"] == 1e-4 and params["solver maxiter"] == 500
    assert "hypre" not in db.values() and not any("hypre" in k for k in db)
    for pre in ("s_", "f_", "p_", "diff_", "fp_fieldsplit_0_"):
        assert db[pre + "pc_type"] == "bjacobi" and db[pre + "sub_pc_type"] == "ilu"
        assert db[pre + "pc_bjacobi_blocks"] == "64"
    # the rest of petsc-options-inexact is untouched
    assert db["fp_pc_fieldsplit_type"] == "schur" and db["fp_pc_fieldsplit_schur_fact_type"] == "lower"
    assert db["fp_pc_fieldsplit_schur_precondition"] == "selfp"
    assert db["fp_fieldsplit_1_pc_type"] == "lu"  # MUMPS -> the device LU (band LU at N=128)
    assert db["s_ksp_type"] == "cg" and db["s_ksp_rtol"] == "1e-1"
    assert db["global_ksp_norm_type"] == "unpreconditioned"


def test_footing_inexact_preset_is_the_reference_set():
    """footing-inexact: footing.py's own inner PC (hypre) with
    petsc-options-inexact unchanged (BoomerAMG settings on every block)."""
    params, db = bench.solver_options(_args("footing-inexact"))
    assert params["solver atol"] == 1e-4 and params["solver maxiter"] == 500
    for pre in ("s_", "f_", "p_", "diff_", "fp_fieldsplit_0_"):
        assert db[pre + "pc_type"] == "hypre"
        assert db[pre + "pc_hypre_boomeramg_coarsen_type"] == "HMIS"
        assert db[pre + "pc_hypre_boomeramg_interp_type"] == "ext+i"
    assert db["fp_fieldsplit_1_pc_type"] == "lu"


def test_fe_cpu_baseline_footing():
    """--system fe with a footing config: the CPU baseline solves the assembled
    footing system (lib/fe_footing.py) and scales by its DoF."""
    from lib.fe_footing import footing_dofs
    a = _args("footing-inexact", system="fe", N=8, cpu_N=4, pc_type="undrained")
    params, db = bench.solver_options(a)
    out = bench.cpu_baseline(a, params, db)
    assert out["value"] > 0 and "footing system" in out["sample"]
    assert abs(out["value"] - out["raw_iters_per_s"] * footing_dofs(4) / footing_dofs(8)) <= 1e-9 * out["value"]


@pytest.mark.parametrize("pc_type", ["diagonal", "diagonal 3-way"])
def test_headline_preset_block_counts(pc_type):
    _, db = bench.solver_options(_args("swelling3d-bjacobi", pc_type=pc_type))
    if pc_type == "diagonal":
        assert db["s_pc_bjacobi_blocks"] == "256" and db["fp_pc_bjacobi_blocks"] == "264"
    else:
        assert db["p_pc_bjacobi_blocks"] == "11" and db["diff_pc_bjacobi_blocks"] == "11"
    assert all(db[p + "ksp_type"] == "preonly" for p in (("s_", "fp_") if pc_type == "diagonal" else
                                                        ("s_", "f_", "p_", "diff_")))


def test_aar_preset():
    args = _args("aar-m5")
    params, _ = bench.solver_options(args)
    assert params["solver type"] == "aar" and params["AAR order"] == 5 and params["AAR p"] == 5


def test_fe_cpu_baseline_runs_the_assembled_system():
    """bench.py --system fe: the CPU baseline solves the assembled swelling
    system (lib/fe_swelling.py) with the preset's options and scales by DoF."""
    a = _args("swelling2d-exact", system="fe", N=8, cpu_N=4)
    params, db = bench.solver_options(a)
    out = bench.cpu_baseline(a, params, db)
    assert out["kind"] == "port" and out["cores"] == 1 and out["value"] > 0
    n4, n8 = 4 * 9 ** 2 + 5 ** 2, 4 * 17 ** 2 + 9 ** 2
    assert abs(out["value"] - out["raw_iters_per_s"] * n4 / n8) <= 1e-9 * out["value"]
    assert "assembled N=4 2-D swelling system" in out["sample"]


@pytest.mark.parametrize("G", [1, 2, 4, 8])
def test_strong_scaling_plan_keeps_the_system(G):
    """--scaling strong (default): the N=59 system and its total block counts
    at every G, so the outer iteration count does not grow with G."""
    a = _args("swelling3d-bjacobi", scaling="strong", replicas=False)
    sharded, N = bench.shard_plan(a, G)
    assert sharded == (G > 1) and N == 59 and (a.blocks_s, a.blocks_fp) == (256, 264)


@pytest.mark.parametrize("G,N", [(2, 74), (4, 94), (8, 118)])
def test_weak_scaling_plan(G, N):
    a = _args("swelling3d-bjacobi", scaling="weak", replicas=False)
    sharded, Ng = bench.shard_plan(a, G)
    assert sharded and Ng == N and (a.blocks_s, a.blocks_fp) == (256 * G, 264 * G)


def test_replicas_plan():
    a = _args("swelling3d-bjacobi", scaling="strong", replicas=True)
    assert bench.shard_plan(a, 4) == (False, 59) and a.scaling == "replicas"


def test_launch_plan_gpus_vs_world_size():
    """--gpus G without WORLD_SIZE launches G ranks itself; inside a job the
    rank count is WORLD_SIZE and a disagreeing --gpus is an error (the driver's
    G-GPU line must never silently run one rank)."""
    assert bench.launch_plan(None, {}) == ("run", 1)
    assert bench.launch_plan(1, {}) == ("run", 1)
    assert bench.launch_plan(8, {}) == ("spawn", 8)
    assert bench.launch_plan(None, {"WORLD_SIZE": "4"}) == ("run", 4)
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}) == ("run", 4)
    assert bench.launch_plan(8, {"WORLD_SIZE": "1"})[0] == "error"
    assert bench.launch_plan(0, {})[0] == "error"


def test_bench_exits_nonzero_on_rank_count_mismatch():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def test_bench_refuses_sharded_ilu():
    """--inner ilu with G > 1 ranks: the library refuses ILU on a sharded block
    as PETSc does (MPIAIJ), so bench exits 2 before launching any rank."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--inner", "ilu"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "redundant_ilu" in r.stderr


def test_bench_records_hypre_semantics():
    import bench
    s = bench.hypre_semantics({"s_pc_type": "hypre"}, 1)
    assert "PMIS" in s["coarsening"] and s["hypre_K"] == 256 and s["relax_min_rows"] == 1024
    assert "np = 3" in bench.hypre_semantics({"pls.hypre_ranks": "3"}, 1)["processes"]
    assert "np = 8 (the sharded" in bench.hypre_semantics({}, 8)["processes"]
    assert bench.hypre_semantics({"pls.hypre_coarsen_chunks": "1"}, 1)["processes"] == "np = 1"
    # default on one rank: BoomerAMG's np = 1 run (no automatic coarsening partitions)
    assert bench.hypre_semantics({"s_pc_type": "hypre"}, 1)["processes"] == "np = 1"
    assert "the most partitions" in bench.hypre_semantics({"pls.hypre_coarsen_chunks": "0"}, 1)["processes"]
