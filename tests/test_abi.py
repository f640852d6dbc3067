"""C-ABI checks that need no GPU: libpls.so loads and exports every entry point
include/pls.h declares; the facade modules import; errors surface as
RuntimeError through pls_last_error."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "pls.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(pls_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "pls_create" in syms and "pls_solve" in syms and len(syms) >= 25


def test_library_exports_every_declared_symbol():
    import lib._native as N
    L = N.lib()
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert set(declared_symbols()) == set(N.EXPORTS)


def test_abi_version_and_error_channel():
    import lib._native as N
    L = N.lib()
    assert L.pls_abi_version() == 1
    # pc type validation happens before any device work
    import lib.handle as H
    with pytest.raises(RuntimeError, match="pc type must be one of"):
        H.Handle.synthetic(2, 2, 1, 0.05, {"pls.pc_type": "bogus"})


def test_facades_import():
    import lib.AAR  # noqa: F401
    import lib.AndersonAcceleration  # noqa: F401
    import lib.IndexSet  # noqa: F401
    import lib.Parser  # noqa: F401
    import lib.Preconditioner  # noqa: F401
    import lib.Solver  # noqa: F401


def test_preconditioner_rejects_bad_pc_type():
    from lib.Preconditioner import Preconditioner
    params = {"pc type": "nope", "inner ksp type": "preonly", "inner pc type": "ilu", "inner rtol": 1e-6,
              "inner atol": 0, "inner maxiter": 10, "inner accel order": 0, "inner monitor": False}
    with pytest.raises(SystemExit, match="pc type must be one of"):
        Preconditioner(None, None, None, None, params, [])
