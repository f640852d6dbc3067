"""Diagnostic: bench.py's --inner hypre configuration at
3-D N=27 sharded over G ranks sharing one GPU (host communicator), histories
saved for a comparison with OracleSolver(dist_size=G) on the CPU
(tools/g8_n27_compare.py).  The G = 1 run with pls.hypre_ranks 8 that round 4
compared against is NOT the same preconditioner: there the fp block's 264
BJACOBI blocks cut the field-major [f | p] rows, while at G = 8 every rank
cuts its own [f_r | p_r] rows into 33 blocks (PETSc's MPIAIJ ownership)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from distutil import launch  # noqa: E402

BOOMER = {"pc_hypre_boomeramg_P_max": "4", "pc_hypre_boomeramg_agg_nl": "1", "pc_hypre_boomeramg_agg_num_paths": "2",
          "pc_hypre_boomeramg_coarsen_type": "HMIS", "pc_hypre_boomeramg_interp_type": "ext+i",
          "pc_hypre_boomeramg_no_CF": "true"}
PARAMS = {"solver type": "gmres", "solver atol": 1e-8, "solver rtol": 1e-6, "solver maxiter": 100,
          "pc type": "diagonal", "inner ksp type": "preonly", "inner pc type": "bjacobi", "inner accel order": 0,
          "AAR order": 10, "AAR p": 5, "AAR omega": 1.0, "AAR beta": 1.0}


def case(N, fp_blocks):
    db = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right", "s_ksp_type": "preonly", "s_pc_type": "hypre",
          "fp_ksp_type": "preonly", "fp_pc_type": "bjacobi", "fp_pc_bjacobi_blocks": str(fp_blocks)}
    db.update({"s_" + k: v for k, v in BOOMER.items()})
    return {"name": f"hypre_n{N}", "dim": 3, "N": N, "params": PARAMS, "db": db}


if __name__ == "__main__":
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 27
    out = os.path.join(ROOT, "gpurun_out", "r5", f"g{G}n{N}")
    os.makedirs(out, exist_ok=True)
    c = case(N, 264)
    if len(sys.argv) > 3 and sys.argv[3] == "solve_first":
        c["solve_first"] = True
        out += "_sf"
        os.makedirs(out, exist_ok=True)
    json.dump(c, open(os.path.join(out, "case.json"), "w"))
    res = launch("gpu", [c], G, out, timeout=1100)
    its = [int(p["its"]) for p in res[c["name"]]]
    print("its per rank", its)
    # keep what the comparison needs (the full per-rank vectors exceed what gpurun copies back)
    import numpy as np
    for r, p in enumerate(res[c["name"]]):
        np.savez(os.path.join(out, f"{c['name']}_rank{r}.npz"), its=p["its"], reason=p["reason"], hist=p["hist"])
