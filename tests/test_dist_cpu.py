"""Multi-process (gloo, world size 2 and 3) checks of the distributed path on CPU.

* The G-rank numpy emulation (oracle/dist.py ``RankSolver2Way``: local rows,
  gathered SpMV input, rank-ordered global sums, block Jacobi inside each
  rank's rows) reproduces the single-process ``OracleSolver(dist_size=G)``:
  same iteration count and reason, every residual-history entry h_k within
  1e-10 h_k + 100 eps h_0 (only the summation order of inner products
  differs; the eps h_0 floor is the rounding of the first residual carried
  down a history that falls 9 orders of magnitude).  This pins the
  oracle that tests/test_dist_gpu.py compares G GPU ranks against.
* The host-staged allgather callback of lib/dist.py (the communicator that lets
  ranks share a GPU) moves bytes in rank order.
* Partition bookkeeping: slabs and per-rank BJACOBI blocks cover every row once.
"""
import numpy as np
import pytest

from distutil import assemble, launch
from oracle import synthetic as S
from oracle.dist import bjacobi_blocks, local_rows, slab
from oracle.solver import OracleSolver

EPS = np.finfo(np.float64).eps

PARAMS = {"solver type": "gmres", "solver atol": 1e-10, "solver rtol": 1e-8, "solver maxiter": 200,
          "pc type": "diagonal", "inner ksp type": "preonly", "inner pc type": "ilu", "inner rtol": 1e-6,
          "inner atol": 0, "inner maxiter": 1000, "inner monitor": False, "solver monitor": False,
          "inner accel order": 0, "AAR order": 10, "AAR p": 5, "AAR omega": 1, "AAR beta": 1}
DB = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right",
      "s_ksp_type": "preonly", "s_pc_type": "bjacobi", "s_pc_bjacobi_blocks": "5",
      "fp_ksp_type": "preonly", "fp_pc_type": "bjacobi", "fp_pc_bjacobi_blocks": "3"}


def _oracle(spec, params, db, G):
    A, P, Pd = S.matrix(spec, 0), S.matrix(spec, 1), S.matrix(spec, 2)
    is_s, is_f, is_p = S.field_major_index_sets(spec)
    return OracleSolver(A, P, Pd, is_s, is_f, is_p, params, db, S.bcs_sub_pressure(spec), dist_size=G)


def test_partition_covers_rows():
    for n, G in ((10, 3), (7, 2), (100, 8), (3, 4)):
        lens = [slab(n, G, r)[1] for r in range(G)]
        assert sum(lens) == n and max(lens) - min(lens) <= 1
    sizes = (50, 50, 13)
    for G in (1, 2, 3):
        rows = np.concatenate([local_rows(sizes, G, r) for r in range(G)])
        assert np.array_equal(np.sort(rows), np.arange(sum(sizes)))
        for fields, nbt in (((0,), 7), ((1, 2), 5), ((2,), 1)):
            blocks = bjacobi_blocks(sizes, fields, G, nbt)
            allb = np.sort(np.concatenate(blocks))
            assert np.array_equal(allb, np.arange(sum(sizes[f] for f in fields)))
            assert len(blocks) == sum(max(1, nbt // G + (1 if r < nbt % G else 0)) for r in range(G))


def test_dist_oracle_g1_is_serial():
    spec = S.SynthSpec(2, 8)
    b = S.rhs(spec)
    o1 = _oracle(spec, PARAMS, DB, 1)
    x1 = o1.solve(b)
    og = _oracle(spec, PARAMS, DB, 1)
    og.block_pc  # same construction path
    assert np.array_equal(og.solve(b), x1)


@pytest.mark.parametrize("world", [2, 3])
def test_rank_emulation_matches_dist_oracle(tmp_path, world):
    case = {"name": f"emul{world}", "dim": 2, "N": 10, "params": PARAMS, "db": DB}
    parts = launch("emul", [case], world, str(tmp_path))[case["name"]]
    spec = S.SynthSpec(2, 10)
    o = _oracle(spec, PARAMS, DB, world)
    xo = o.solve(S.rhs(spec))
    ho = np.asarray(o.history)
    for p in parts:
        assert int(p["its"]) == o.its and int(p["reason"]) == o.reason
        assert np.all(np.abs(p["hist"] - ho) <= 1e-10 * ho + 100 * EPS * ho[0])
    x = assemble(parts)
    assert np.allclose(x, xo, rtol=1e-10, atol=1e-12 * np.abs(xo).max())
    # the G-rank preconditioner differs from the serial one (blocks per rank)
    o1 = _oracle(spec, PARAMS, DB, 1)
    o1.solve(S.rhs(spec))
    assert not np.allclose(np.asarray(o1.history)[:len(ho)][:5], ho[:5], rtol=1e-12, atol=0)


def test_host_callback_allgather(tmp_path):
    case = {"name": "cb", "bytes": 37}
    parts = launch("callback", [case], 2, str(tmp_path))["cb"]
    expect = np.concatenate([[(r * 7 + j) % 256 for j in range(37)] for r in range(2)]).astype(np.uint8)
    for p in parts:
        assert int(p["rc"]) == 0
        assert np.array_equal(p["recv"], expect)
