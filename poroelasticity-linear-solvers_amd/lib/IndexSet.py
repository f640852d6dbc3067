"""Field index sets (reference lib/IndexSet.py:29-67), contract only.

The reference builds them from dolfin dofmaps; here they are built from plain
integer arrays (the dofmap ``dofs()`` of each sub-space).  In 2-way mode is_f /
is_p are re-indexed to their positions inside the sorted fp set, exactly as
``get_local_fp_dofs`` does (IndexSet.py:10-26,46-54).
"""
from time import perf_counter as time

import numpy as np

from .Printing import parprint


class IS:
    """Minimal stand-in for a PETSc IS: ``getIndices`` / ``getSize`` / len."""

    def __init__(self, indices):
        self._idx = np.ascontiguousarray(np.asarray(indices), dtype=np.int32)

    def getIndices(self):
        return self._idx

    def getSize(self):
        return int(self._idx.size)

    def __len__(self):
        return int(self._idx.size)


def get_local_fp_dofs(dofs_fp_global, dofmap_f, dofmap_p):
    """Positions of the f and p dofs inside the sorted fp dof list."""
    dofs_fp_global = np.asarray(dofs_fp_global)
    in_f = np.isin(dofs_fp_global, np.asarray(dofmap_f))
    in_p = np.isin(dofs_fp_global, np.asarray(dofmap_p)) & ~in_f
    pos = np.arange(dofs_fp_global.size, dtype=np.int32)
    return pos[in_f], pos[in_p]


class IndexSet:
    """``IndexSet(V, two_way)``: V is a dolfin mixed FunctionSpace (as in the
    reference) or a tuple ``(dofs_s, dofs_f, dofs_p)`` of integer arrays."""

    def __init__(self, V, two_way=True):
        t0 = time()
        if hasattr(V, "sub"):
            dofs_s, dofs_f, dofs_p = (V.sub(i).dofmap().dofs() for i in range(3))
        else:
            dofs_s, dofs_f, dofs_p = V
        self.dofmap_s = np.asarray(dofs_s, dtype=np.int64)
        self.dofmap_f = np.asarray(dofs_f, dtype=np.int64)
        self.dofmap_p = np.asarray(dofs_p, dtype=np.int64)
        self.ns, self.nf, self.np = int(self.dofmap_s.size), int(self.dofmap_f.size), int(self.dofmap_p.size)
        self.global_f, self.global_p = self.dofmap_f.copy(), self.dofmap_p.copy()
        self.dofmap_fp = np.sort(np.concatenate([self.dofmap_f, self.dofmap_p]))
        self.two_way = two_way
        if two_way:
            # IndexSet.py:44-54: positions inside the all-gathered global fp list
            dofs_fp_global = self.dofmap_fp
            from .dist import world
            if world()[1] > 1:
                import torch.distributed as td
                parts = [None] * world()[1]
                td.all_gather_object(parts, self.dofmap_fp.tolist())
                dofs_fp_global = np.asarray([d for part in parts for d in part], dtype=np.int64)
            self.dofmap_f, self.dofmap_p = get_local_fp_dofs(dofs_fp_global, self.dofmap_f, self.dofmap_p)
        self.is_s = IS(self.dofmap_s)
        self.is_f = IS(self.dofmap_f)
        self.is_p = IS(self.dofmap_p)
        self.is_fp = IS(self.dofmap_fp)
        parprint("---- [Indexes] computed local indices in {:.3f}s".format(time() - t0))

    def get_dimensions(self):
        return self.ns, self.nf, self.np

    def get_index_sets(self):
        return self.is_s, self.is_f, self.is_p, self.is_fp

    def global_index_sets(self):
        """(is_s, is_f, is_p) as global sorted indices (what libpls needs)."""
        return (np.ascontiguousarray(self.dofmap_s, dtype=np.int32),
                np.ascontiguousarray(self.global_f, dtype=np.int32),
                np.ascontiguousarray(self.global_p, dtype=np.int32))
