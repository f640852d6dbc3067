"""PETSc binary Mat/Vec/IS reader-writer (lib/petsc_io.py).

Known answer: a file assembled byte by byte from PETSc's documented binary
layout (big-endian int32 classid / sizes / row lengths / columns, float64
values).  Plus round trips, multi-object files and malformed input.  A GPU
test (test_gpu_parity-style) solves a system loaded from such files.
"""
import struct

import numpy as np
import pytest
import scipy.sparse as sp

from lib import petsc_io as pio


def test_known_answer_mat_bytes(tmp_path):
    # [[1, 0, 2], [0, 0, 3]] : rows of length 2 and 1
    raw = struct.pack(">4i", 1211216, 2, 3, 3) + struct.pack(">2i", 2, 1) + struct.pack(">3i", 0, 2, 2) + \
        struct.pack(">3d", 1.0, 2.0, 3.0)
    f = tmp_path / "m.bin"
    f.write_bytes(raw)
    M = pio.read_mat(str(f))
    assert M.shape == (2, 3)
    assert np.array_equal(M.toarray(), [[1.0, 0.0, 2.0], [0.0, 0.0, 3.0]])
    pio.write_mat(str(tmp_path / "w.bin"), M)
    assert (tmp_path / "w.bin").read_bytes() == raw


def test_known_answer_vec_and_is(tmp_path):
    raw = struct.pack(">2i", 1211214, 3) + struct.pack(">3d", 0.5, -1.0, 2.25) + \
        struct.pack(">2i", 1211218, 2) + struct.pack(">2i", 7, 4)
    f = tmp_path / "v.bin"
    f.write_bytes(raw)
    objs = pio.read_objects(str(f))
    assert [k for k, _ in objs] == ["vec", "is"]
    assert np.array_equal(objs[0][1], [0.5, -1.0, 2.25]) and np.array_equal(objs[1][1], [7, 4])


def test_round_trip_multi_object(tmp_path):
    rng = np.random.default_rng(0)
    A = sp.random(50, 40, density=0.1, random_state=rng, format="csr")
    v = rng.standard_normal(17)
    iset = rng.permutation(30).astype(np.int32)
    f = str(tmp_path / "all.bin")
    pio.write_objects(f, [("mat", A), ("vec", v)])
    pio.write_is(f, iset, append=True)
    objs = pio.read_objects(f)
    assert [k for k, _ in objs] == ["mat", "vec", "is"]
    assert (objs[0][1] != A).nnz == 0 and np.array_equal(objs[1][1], v) and np.array_equal(objs[2][1], iset)


def test_malformed(tmp_path):
    f = tmp_path / "bad.bin"
    f.write_bytes(struct.pack(">4i", 1211216, 2, 2, 5) + struct.pack(">2i", 1, 1))
    with pytest.raises(pio.PetscBinaryError, match="truncated"):
        pio.read_mat(str(f))
    f.write_bytes(struct.pack(">2i", 42, 0))
    with pytest.raises(pio.PetscBinaryError, match="classid"):
        pio.read_objects(str(f))
    f.write_bytes(struct.pack(">4i", 1211216, 2, 2, 3) + struct.pack(">2i", 1, 1) + struct.pack(">3i", 0, 1, 1) +
                  struct.pack(">3d", 1, 2, 3))
    with pytest.raises(pio.PetscBinaryError, match="sum"):
        pio.read_mat(str(f))


@pytest.mark.gpu
def test_solve_from_petsc_binary_files(gpu, tmp_path):
    """A, P, P_diff, index sets and b written as PETSc binary files, loaded and
    solved through Handle.from_csr: identical to the in-HBM synthetic handle."""
    from lib.handle import Handle, params_to_options
    from oracle import synthetic as S
    spec = S.SynthSpec(2, 9)
    is_s, is_f, is_p = S.field_major_index_sets(spec)
    f = str(tmp_path / "system.bin")
    pio.write_objects(f, [("mat", S.matrix(spec, 0)), ("mat", S.matrix(spec, 1)), ("mat", S.matrix(spec, 2)),
                          ("is", is_s), ("is", is_f), ("is", is_p), ("vec", S.rhs(spec))])
    (_, A), (_, P), (_, Pd), (_, s), (_, fi), (_, p), (_, b) = pio.read_objects(f)
    params = {"solver type": "gmres", "solver atol": 1e-10, "solver rtol": 1e-8, "solver maxiter": 200,
              "pc type": "diagonal 3-way", "inner ksp type": "preonly", "inner pc type": "ilu"}
    opts = {"global_ksp_type": "gmres", "global_ksp_pc_side": "right"}
    for pre in ("s_", "f_", "p_", "diff_"):
        opts[pre + "ksp_type"] = "preonly"
        opts[pre + "pc_type"] = "ilu"
    opts.update(params_to_options(params))
    hf = Handle.from_csr(A, P, Pd, s, fi, p, S.bcs_sub_pressure(spec), opts)
    hs = Handle.synthetic(spec.dim, spec.N, spec.seed, spec.delta, opts)
    xf, rf = hf.solve(b)
    xs, rs = hs.solve(b)
    assert rf.its == rs.its and np.array_equal(hf.history(), hs.history()) and np.array_equal(xf, xs)
