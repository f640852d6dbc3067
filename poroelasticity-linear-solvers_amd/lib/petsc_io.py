"""PETSc binary files: read / write Mat (AIJ), Vec and IS objects.

Lets matrices and vectors dumped from the reference run -- e.g. with
``PETSc.Viewer().createBinary(path, "w")`` and ``A.mat().view(viewer)`` inside
``lib/Poromechanics.py`` after assembly -- feed
``Handle.from_csr`` / ``Solver`` here on a machine without PETSc.

Format (PETSc's MatView/VecView/ISView binary, default 32-bit indices,
real double scalars, big-endian):

* Mat: int32 classid 1211216, M, N, nz, int32 row_lengths[M],
  int32 col_indices[nz], float64 values[nz]  (rows in order, columns as stored);
* Vec: int32 classid 1211214, n, float64 values[n];
* IS:  int32 classid 1211218, n, int32 indices[n].

Objects are stored back to back; ``read_objects`` walks a file.
"""
from __future__ import annotations

import numpy as np

MAT_FILE_CLASSID = 1211216
VEC_FILE_CLASSID = 1211214
IS_FILE_CLASSID = 1211218

_I4, _F8 = np.dtype(">i4"), np.dtype(">f8")


class PetscBinaryError(ValueError):
    pass


def _take(buf, off, dtype, count):
    end = off + dtype.itemsize * count
    if end > len(buf):
        raise PetscBinaryError(f"truncated file: need {end} bytes, have {len(buf)}")
    return np.frombuffer(buf, dtype=dtype, count=count, offset=off), end


def _read_one(buf, off):
    (cid,), off = _take(buf, off, _I4, 1)
    if cid == MAT_FILE_CLASSID:
        (m, n, nz), off = _take(buf, off, _I4, 3)
        if m < 0 or n < 0 or nz < 0:
            raise PetscBinaryError("negative Mat header sizes (64-bit-index files are not supported)")
        lens, off = _take(buf, off, _I4, m)
        cols, off = _take(buf, off, _I4, nz)
        vals, off = _take(buf, off, _F8, nz)
        lens = lens.astype(np.int64)
        if lens.sum() != nz:
            raise PetscBinaryError("row lengths do not sum to nz")
        rp = np.zeros(m + 1, dtype=np.int64)
        np.cumsum(lens, out=rp[1:])
        import scipy.sparse as sp
        M = sp.csr_matrix((vals.astype(np.float64), cols.astype(np.int32), rp), shape=(int(m), int(n)))
        return ("mat", M), off
    if cid == VEC_FILE_CLASSID:
        (n,), off = _take(buf, off, _I4, 1)
        v, off = _take(buf, off, _F8, n)
        return ("vec", v.astype(np.float64)), off
    if cid == IS_FILE_CLASSID:
        (n,), off = _take(buf, off, _I4, 1)
        v, off = _take(buf, off, _I4, n)
        return ("is", v.astype(np.int32)), off
    raise PetscBinaryError(f"unknown PETSc classid {cid} at byte {off - 4}")


def read_objects(path):
    """All objects of a PETSc binary file, in order: [(kind, object), ...]."""
    with open(path, "rb") as fh:
        buf = fh.read()
    out, off = [], 0
    while off < len(buf):
        obj, off = _read_one(buf, off)
        out.append(obj)
    return out


def _first(path, kind):
    for k, o in read_objects(path):
        if k == kind:
            return o
    raise PetscBinaryError(f"no {kind} object in {path}")


def read_mat(path):
    """First Mat of the file as a scipy CSR matrix (MatLoad)."""
    return _first(path, "mat")


def read_vec(path):
    return _first(path, "vec")


def read_is(path):
    return _first(path, "is")


def _mat_bytes(M):
    import scipy.sparse as sp
    M = sp.csr_matrix(M)
    m, n = M.shape
    lens = np.diff(M.indptr).astype(_I4)
    head = np.array([MAT_FILE_CLASSID, m, n, M.nnz], dtype=_I4)
    return (head.tobytes() + lens.tobytes() + M.indices.astype(_I4).tobytes() +
            M.data.astype(_F8).tobytes())


def write_objects(path, objects, append=False):
    """objects: [("mat", csr) | ("vec", array) | ("is", array), ...] (MatView/VecView/ISView)."""
    with open(path, "ab" if append else "wb") as fh:
        for kind, o in objects:
            if kind == "mat":
                fh.write(_mat_bytes(o))
            elif kind == "vec":
                v = np.asarray(o, dtype=_F8)
                fh.write(np.array([VEC_FILE_CLASSID, v.size], dtype=_I4).tobytes() + v.tobytes())
            elif kind == "is":
                v = np.asarray(o, dtype=_I4)
                fh.write(np.array([IS_FILE_CLASSID, v.size], dtype=_I4).tobytes() + v.tobytes())
            else:
                raise ValueError(f"unknown object kind {kind!r}")


def write_mat(path, M, append=False):
    write_objects(path, [("mat", M)], append)


def write_vec(path, v, append=False):
    write_objects(path, [("vec", v)], append)


def write_is(path, v, append=False):
    write_objects(path, [("is", v)], append)
