"""P2-P2-P1 assembly of the footing problem (footing.py, 2-D; numpy).

configs[2] of BASELINE.json names ``footing.py``; this module produces its
true first-time-step system -- A, P, P_diff, b, index sets, pressure-BC
positions -- the way ``lib/fe_swelling.py`` does for the swelling drivers
(SURVEY.md 8(f) rank 2).  An input generator: nothing in the solve path
imports it.

What it restates (no dolfin here):

* mesh (``lib/MeshCreation.py:53-77``): ``UnitSquareMesh(N, N)`` ("right"
  diagonal) scaled by ``length`` = 64 (``footing.py:17-19``), then refined
  twice where a cell lies in the top third away from the sides (vertex
  y_min > 2L/3, x_min > L/8, x_max < 7L/8; ``MeshCreation.py:59-72``) by
  dolfin's default local refinement, the Plaza algorithm
  (``PlazaRefinementND``): the edges of marked cells are marked, then every
  cell with a marked edge marks its longest edge until nothing changes (a
  conforming mesh), each cell is split by bisection of its longest edge plus
  its other marked edges -- or, when all three edges are marked and the
  shortest/longest edge ratio is >= sqrt(2)/2, into the four "red"
  children; ``refinements`` further uniform (red) refinements
  (``MeshCreation.py:76-77``);
* parameters ``footing.py:42-89`` (E = 3e4, nu = 0.2, ...; "pc type"
  undrained), forms of ``lib/Assembler.py`` via ``fe_swelling.assemble_forms``;
* right-hand side at the first step t = dt: the solid traction
  ``fs_sur = (0, |x - L/2| < L/4 ? -min(t, 1) 1e5 : 0)`` (an ``Expression`` of
  degree 1, i.e. its P1 interpolant) on the TOP facets (``footing.py:22-24,
  37-39``); no other loads;
* Dirichlet conditions (``footing.py:97-111``): solid u = 0 on BOTTOM;
  fluid v = 0 on the foot (top boundary facets with every vertex and the
  midpoint in |x - L/2| < L/4); pressure p = 0 (P_diff only) on every other
  boundary facet -- dolfin's ``SubDomain.mark`` rule (all vertices and the
  midpoint inside) with the topological DirichletBC method.

Dof numbering is this module's own (RCM over P2 nodes), as in
``fe_swelling``.  The mesh is pinned by its geometry (area, conformity,
counts), not against dolfin (absent): parity of the mesh is unpinned.
"""
from __future__ import annotations

import numpy as np

from . import fe_swelling as F

LENGTH = 64.0
_E, _NU = 3e4, 0.2
# footing.py:42-66
FOOTING = dict(mu_f=1e-3, rhof=1e3, rhos=500.0, phi0=1e-3, mu_s=_E / (2 * (1 + _NU)),
               lmbda=_E * _NU / ((1 + _NU) * (1 - 2 * _NU)), ks=1e6, kf=1e-7, dt=0.1, betas=-0.5, betaf=0.0,
               betap=1.0)
_EPS = 3e-16  # DOLFIN_EPS of near()


def _edges(cells):
    """Unique edges (sorted vertex pairs) and the cell -> edge map, local edge
    i opposite local vertex i."""
    nc = cells.shape[0]
    le = np.stack([np.sort(cells[:, [(i + 1) % 3, (i + 2) % 3]], 1) for i in range(3)], 1)
    uniq, inv = np.unique(le.reshape(-1, 2), axis=0, return_inverse=True)
    return uniq, inv.reshape(nc, 3)


def plaza_refine(coords, cells, cell_marked):
    """One Plaza refinement of a triangle mesh (dolfin's default local
    refinement; see the module docstring).  Returns (coords, cells)."""
    nv, nc = coords.shape[0], cells.shape[0]
    uniq, c2e = _edges(cells)
    d = coords[uniq[:, 1]] - coords[uniq[:, 0]]
    elen = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1])
    L = elen[c2e]
    longest = np.argmax(L, 1)  # local index of the longest edge (= its opposite vertex)
    ratio_ok = L.min(1) / L.max(1) >= np.sqrt(2.0) / 2.0
    marked = np.zeros(uniq.shape[0], bool)
    marked[c2e[np.asarray(cell_marked, bool)].ravel()] = True
    ar = np.arange(nc)
    lidx = c2e[ar, longest]
    while True:  # conformity: a cell with any marked edge bisects its longest edge
        need = marked[c2e].any(1) & ~marked[lidx]
        if not need.any():
            break
        marked[lidx[need]] = True
    mid = np.full(uniq.shape[0], -1, dtype=np.int64)
    mid[marked] = nv + np.arange(int(marked.sum()))
    new_coords = np.concatenate([coords, 0.5 * (coords[uniq[marked, 0]] + coords[uniq[marked, 1]])])

    out = [cells[~marked[c2e].any(1)]]
    for c in np.nonzero(marked[c2e].any(1))[0]:
        le = longest[c]
        i0, i1, i2 = (le + 1) % 3, (le + 2) % 3, le
        v0, v1, v2 = cells[c, i0], cells[c, i1], cells[c, i2]
        e0, e1, e2 = mid[c2e[c, i0]], mid[c2e[c, i1]], mid[c2e[c, i2]]
        m0, m1 = marked[c2e[c, i0]], marked[c2e[c, i1]]
        if ratio_ok[c] and m0 and m1:
            t = [(e0, e1, v2), (e1, e2, v0), (e2, e0, v1), (e2, e1, e0)]
        else:
            t = [(e2, v2, e0), (e2, e0, v1)] if m0 else [(e2, v2, v1)]
            t += [(e2, v2, e1), (e2, e1, v0)] if m1 else [(e2, v2, v0)]
        out.append(np.array(t, dtype=np.int64))
    return new_coords, np.concatenate(out)


def footing_mesh(N: int, length: float = LENGTH, refinements: int = 0):
    """generate_footing_square (MeshCreation.py:53-77): float vertex
    coordinates (nv x 2) and triangles (nc x 3)."""
    icoords, cells = F.unit_mesh(2, N)
    # UnitSquareMesh's vertices are i / N, then coordinates *= length (ADVICE r02:
    # i * (length / N) misses the top edge by an ulp for some N, e.g. 49)
    coords = (icoords.astype(np.float64) / N) * length
    for _ in range(2):
        x, y = coords[cells, 0], coords[cells, 1]
        mark = (y.min(1) > 2 * length / 3) & (x.min(1) > length / 8) & (x.max(1) < 7 / 8 * length)
        coords, cells = plaza_refine(coords, cells, mark)
    for _ in range(refinements):
        coords, cells = plaza_refine(coords, cells, np.ones(cells.shape[0], bool))
    return coords, cells


def footing_dofs(N: int, refinements: int = 0) -> int:
    """Size of the footing system (P2-P2-P1 on the refined mesh)."""
    c, cells = footing_mesh(N, LENGTH, refinements)
    return 4 * (c.shape[0] + _edges(cells)[0].shape[0]) + c.shape[0]


def boundary_facets(cells):
    """Edges (vertex pairs) that belong to exactly one cell, and the P2 node
    number of each (nv + edge index in the unique-edge order used by
    :func:`p2_nodes`)."""
    uniq, c2e = _edges(cells)
    cnt = np.bincount(c2e.ravel(), minlength=uniq.shape[0])
    b = np.nonzero(cnt == 1)[0]
    return uniq[b], b


def p2_nodes(coords, cells):
    """P2 nodes: vertices, then the unique edges.  cell_nodes lists a cell's
    vertices then its edges in itertools.combinations order (the order
    fe_swelling's element blocks assume)."""
    nv, nc = coords.shape[0], cells.shape[0]
    pairs = [(0, 1), (0, 2), (1, 2)]
    e = np.stack([np.sort(cells[:, [a, b]], 1) for a, b in pairs], 1)
    uniq, c2e = _edges(cells)
    # edge number of each (cell, pair) in the unique order of _edges
    key = uniq[:, 0] * (nv + 1) + uniq[:, 1]
    k = e[..., 0] * (nv + 1) + e[..., 1]
    eidx = np.searchsorted(key, k.ravel()).reshape(nc, 3)
    cell_nodes = np.concatenate([cells, nv + eidx], 1)
    xnode = np.concatenate([coords, 0.5 * (coords[uniq[:, 0]] + coords[uniq[:, 1]])])
    return cell_nodes, xnode, uniq


def assemble_footing(N: int, pc_type: str = "undrained", params: dict | None = None, ordering: str = "field-major",
                     t: float | None = None, refinements: int = 0, length: float = LENGTH) -> F.SwellingSystem:
    """The footing system at the first time step (footing.py + lib/Poromechanics.py:58-98)."""
    prm = dict(FOOTING, **(params or {}))
    t = prm["dt"] if t is None else t
    coords, cells = footing_mesh(N, length, refinements)
    nv = coords.shape[0]
    cell_nodes, xnode, uniq = p2_nodes(coords, cells)
    nnodes = xnode.shape[0]
    A, P, Pd, (us, vf, p) = F.assemble_forms(2, coords[cells], cells, cell_nodes, nv, nnodes, pc_type, prm, ordering)
    n = A.shape[0]

    bf, bnode = boundary_facets(cells)
    bnode = nv + bnode  # the facet's edge node
    xa, xb, xm = coords[bf[:, 0]], coords[bf[:, 1]], xnode[bnode]

    def on_all(pred):  # SubDomain.mark: every vertex and the midpoint inside
        return pred(xa) & pred(xb) & pred(xm)

    def near(a, b):
        return np.abs(a - b) < _EPS

    top = on_all(lambda x: near(x[:, 1], length))
    if not top.any():
        raise ValueError(f"footing mesh N={N}: no facet on the top edge (traction and foot BCs would be lost)")
    bottom = on_all(lambda x: near(x[:, 1], 0.0))
    foot = on_all(lambda x: near(x[:, 1], length) & (np.abs(x[:, 0] - length / 2) < length / 4))
    not_foot = on_all(lambda x: ~(near(x[:, 1], length) & (np.abs(x[:, 0] - length / 2) < length / 4)))

    # ---- right-hand side: P1 interpolant of fs_sur on the TOP facets (footing.py:37-39):
    # int (g0 l0 + g1 l1) phi: vertex a -> g_a |e| / 6, edge node -> (g0 + g1) |e| / 3
    val = min(t, 1.0) * 1e5
    L2 = length / 2

    def g(x):
        return np.where(np.abs(x[:, 0] - L2) < L2 / 2, -val, 0.0)

    b = np.zeros(n)
    ft = np.nonzero(top)[0]
    ell = np.linalg.norm(xb[ft] - xa[ft], axis=1)
    ga, gb = g(xa[ft]), g(xb[ft])
    np.add.at(b, us[bf[ft, 0], 1], ga * ell / 6)
    np.add.at(b, us[bf[ft, 1], 1], gb * ell / 6)
    np.add.at(b, us[bnode[ft], 1], (ga + gb) * ell / 3)

    def facet_nodes(sel):
        idx = np.nonzero(sel)[0]
        return np.unique(np.concatenate([bf[idx, 0], bf[idx, 1], bnode[idx]]))

    bc_rows = np.unique(np.concatenate([us[facet_nodes(bottom)].ravel(), vf[facet_nodes(foot)].ravel()]))
    pv = facet_nodes(not_foot)
    p_rows = np.unique(p[pv[pv < nv]])
    A, P = F._dirichlet(A, bc_rows), F._dirichlet(P, bc_rows)
    b[bc_rows] = 0.0
    if Pd is not None:
        Pd = F._dirichlet(F._dirichlet(Pd, bc_rows), p_rows)
    is_s, is_f, is_p = (np.sort(x.ravel()).astype(np.int32) for x in (us, vf, p))
    bcs_sub = np.searchsorted(is_p, p_rows).astype(np.int32)
    return F.SwellingSystem(A, P, Pd, b, is_s, is_f, is_p, bcs_sub, 2, N)
