"""Host side of the reference-harness restatement (tools/robustness.py): the
option files parse as the reference's Parser does, mpirun -np 8's BoomerAMG
semantics map to the library options, the driver parameter sets are
swelling.py's / footing.py's, and the results table renders."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_option_sets_parse():
    import robustness as R
    ex = R.load_set("exact")
    assert ex["global_ksp_pc_side"] == "right" and ex["s_pc_type"] == "lu" and ex["fp_pc_type"] == "lu"
    inx = R.load_set("inexact")
    # petsc-options-inexact:4-5 (no pc side: unpreconditioned norm), 10-24, 73-106
    assert "global_ksp_pc_side" not in inx and inx["global_ksp_norm_type"] == "unpreconditioned"
    assert inx["s_ksp_type"] == "cg" and inx["s_ksp_rtol"] == "1e-1" and inx["s_pc_type"] == "hypre"
    assert inx["s_pc_hypre_boomeramg_no_CF"] == "true" and inx["s_pc_hypre_boomeramg_P_max"] == "4"
    assert inx["fp_pc_fieldsplit_schur_precondition"] == "selfp" and inx["fp_fieldsplit_0_ksp_max_it"] == "10"
    assert inx["fp_fieldsplit_1_pc_type"] == "lu" and inx["diff_ksp_type"] == "preonly"


def test_np8_semantics_and_drivers():
    import robustness as R
    assert R.np_options(8) == {"pls.hypre_ranks": "8", "pls.hypre_relax_chunks": "8"}
    assert R.np_options(1) == {"pls.hypre_relax_chunks": "1"}
    # swelling.py:62-66, footing.py:66-70
    assert R.DRIVER["swelling"]["solver atol"] == 1e-8 and R.DRIVER["footing"]["solver atol"] == 1e-4
    for d in R.DRIVER.values():
        assert d["solver rtol"] == 1e-6 and d["solver maxiter"] == 500 and d["inner pc type"] == "hypre"


def test_table_renders(tmp_path):
    row = {"problem": "footing", "N": 10, "pc_type": "undrained", "options": "inexact", "np": 8, "dofs": 7857,
           "nnz": 1, "its": 36, "reason": 2, "rnorm0": 1.0, "rnorm": 9e-7, "assembly_s": 0.1, "setup_s": 0.2,
           "solve_s": 0.07, "inner": {"s_": {"solves": 37, "its": 248, "max": 8, "negative_reason": 0}}, "extra": {}}
    f = tmp_path / "r.jsonl"
    f.write_text(json.dumps(row) + "\n" + json.dumps(dict(row, reason=-100)) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "robustness_table.py"), str(f)],
                         capture_output=True, text=True, check=True).stdout
    lines = [ln for ln in out.splitlines() if ln.startswith("| footing")]
    assert len(lines) == 1 and "time limit" in lines[0] and "s 248 (7 / 8)" in lines[0]
