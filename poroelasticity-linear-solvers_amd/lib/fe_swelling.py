"""P2-P2-P1 finite-element assembly of the swelling test problem (numpy).

Produces true poromechanics systems -- A, P, P_diff, b, the field index sets
and the pressure-BC positions -- in the form the reference hands across the
solver boundary, so the solver can be exercised on the saddle-point operators
the reference drivers build rather than only on the random SPD blocks of
SURVEY.md 8(d) ("a numpy structured P2-P2-P1
assembler").  This is an input generator: nothing in the solve path imports it.

What it restates (no dolfin here; the forms are integrated directly):

* mesh: ``UnitSquareMesh(N, N)`` ("right" diagonal) / ``UnitCubeMesh(N, N, N)``
  (the six Kuhn tetrahedra around each cube's main diagonal), scaled by the
  side length 1e-2 (``lib/MeshCreation.py:11-20,169-178``);
* space: vector P2 solid displacement, vector P2 fluid velocity, P1 pressure
  (``lib/Poromechanics.py:14-18``); the sparsity is the full mixed-element cell
  coupling (every dof of a cell couples with every dof of the cell), shared by
  A, P and P_diff, explicit zeros kept -- dolfin's pattern;
* forms: the base matrix A and the preconditioner matrices P / P_diff of every
  ``pc type`` branch (``lib/Assembler.py:66-221``), constant coefficients;
* right-hand side: the surface tractions of the first time step, t = dt
  (``lib/Assembler.py:235-269``; only ``rhs_*`` terms reach ``b``; zero volume
  loads and pressure source, ``swelling.py:28-39``, ``swelling-3d.py:28-39``);
* Dirichlet conditions: dolfin ``DirichletBC.apply`` -- bc rows zeroed with a
  unit diagonal in A, P (and P_diff), bc entries of b set to 0; the pressure
  BCs go to P_diff only, and their positions inside the pressure sub-vector
  are ``bcs_sub_pressure`` (``lib/Poromechanics.py:40-55,72-83``;
  ``swelling.py:93-104``; ``swelling-3d.py:95-107``).

Dof numbering is this module's own (dolfin's dof order cannot be reproduced
without dolfin): P2 nodes in reverse Cuthill-McKee order, either
``field-major`` (all u_s, then all v_f, then p) or ``interleaved`` (per node:
u_s components, v_f components, then p if the node is a vertex -- dolfin-like,
the fields are then picked out by the index sets).
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import reverse_cuthill_mckee

# swelling.py:41-52 / swelling-3d.py:43-63 (ks differs)
SWELLING_2D = dict(mu_f=0.035, rhof=1e3, rhos=1e3, phi0=0.1, mu_s=4000.0, lmbda=700.0, ks=1e6, kf=1e-7,
                   dt=0.1, betas=-0.5, betaf=0.0, betap=1.0)
SWELLING_3D = dict(SWELLING_2D, ks=1e8)
SIDE_LENGTH = 1e-2

PC_TYPES = ("undrained", "undrained 3-way", "diagonal", "diagonal 3-way", "diagonal 3-way-II")


@dataclass
class SwellingSystem:
    A: sp.csr_matrix
    P: sp.csr_matrix
    P_diff: sp.csr_matrix | None
    b: np.ndarray
    is_s: np.ndarray
    is_f: np.ndarray
    is_p: np.ndarray
    bcs_sub_pressure: np.ndarray
    dim: int
    N: int

    @property
    def dims(self):
        return self.is_s.size, self.is_f.size, self.is_p.size


# ------------------------------------------------------------------ mesh --
def unit_mesh(dim: int, N: int):
    """Integer vertex grid coordinates (nv x dim) and simplices (nc x dim+1).
    Vertex (i, j[, k]) has index i + (N+1) j [+ (N+1)^2 k]; each square/cube is
    split into the Kuhn simplices v0, v0+e_a, v0+e_a+e_b, ... over every axis
    permutation -- the 2 / 6 cells of dolfin's UnitSquareMesh ("right") /
    UnitCubeMesh."""
    n1 = N + 1
    strides = [n1 ** a for a in range(dim)]
    base = np.meshgrid(*([np.arange(N)] * dim), indexing="ij")
    v0 = sum(base[a].ravel() * strides[a] for a in range(dim))
    cells = []
    for perm in itertools.permutations(range(dim)):
        verts, cur = [v0], v0
        for a in perm:
            cur = cur + strides[a]
            verts.append(cur)
        cells.append(np.stack(verts, 1))
    cells = np.concatenate(cells)
    flat = np.arange(n1 ** dim)
    coords = np.stack([(flat // strides[a]) % n1 for a in range(dim)], 1)
    return coords.astype(np.int64), cells.astype(np.int64)


def _p2_nodes(dim, N):
    coords, cells = unit_mesh(dim, N)
    nv = coords.shape[0]
    pairs = list(itertools.combinations(range(dim + 1), 2))
    e = np.stack([np.sort(cells[:, [a, b]], 1) for a, b in pairs], 1)  # nc x ne x 2
    uniq, inv = np.unique(e.reshape(-1, 2), axis=0, return_inverse=True)
    cell_nodes = np.concatenate([cells, nv + inv.reshape(cells.shape[0], len(pairs))], 1)
    node2x = np.concatenate([2 * coords, coords[uniq[:, 0]] + coords[uniq[:, 1]]])  # doubled grid coords
    return coords, cells, pairs, cell_nodes, node2x, nv


# ------------------------------------------------------------ quadrature --
def _simplex_rule(dim, n=4):
    """Collapsed (Duffy) Gauss-Legendre rule on the reference simplex, exact
    beyond degree 4 (the P2 x P2 mass integrand)."""
    g, w = np.polynomial.legendre.leggauss(n)
    g, w = 0.5 * (g + 1), 0.5 * w
    pts, wts = [], []
    for ii in itertools.product(range(n), repeat=dim):
        u = [g[i] for i in ii]
        ww = np.prod([w[i] for i in ii])
        xi, scale = [], 1.0
        for a in range(dim):
            xi.append(u[a] * scale)
            ww *= scale if a > 0 else 1.0
            scale *= (1 - u[a])
        pts.append(xi)
        wts.append(ww)
    return np.array(pts), np.array(wts)


def _p2_basis(dim, pts, pairs):
    """Values (nq x nb) and reference gradients (nq x nb x dim) of the P2
    basis: vertex i -> l_i(2 l_i - 1), edge (i, j) -> 4 l_i l_j."""
    lam = np.concatenate([1 - pts.sum(1, keepdims=True), pts], 1)
    dlam = np.concatenate([-np.ones((1, dim)), np.eye(dim)])  # (dim+1) x dim
    vals = [lam[:, i] * (2 * lam[:, i] - 1) for i in range(dim + 1)]
    grads = [(4 * lam[:, i] - 1)[:, None] * dlam[i] for i in range(dim + 1)]
    for i, j in pairs:
        vals.append(4 * lam[:, i] * lam[:, j])
        grads.append(4 * (lam[:, i][:, None] * dlam[j] + lam[:, j][:, None] * dlam[i]))
    return np.stack(vals, 1), np.stack(grads, 1), lam, dlam


# ------------------------------------------------------- element blocks --
def _element_blocks(dim, xcells):
    """Per-cell elementary matrices (physical coordinates, constant J):
    M2 (P2 mass), G[a,b,k,l] = int d_k phi_a d_l phi_b, C[e,a,k] =
    int psi_e d_k phi_a (psi = P1), Mp, Kp (P1 mass / stiffness)."""
    pts, wts = _simplex_rule(dim)
    pairs = list(itertools.combinations(range(dim + 1), 2))
    phi, dphi, lam, dlam = _p2_basis(dim, pts, pairs)
    J = np.stack([xcells[:, a + 1] - xcells[:, 0] for a in range(dim)], 2)  # nc x dim x dim (columns)
    det = np.abs(np.linalg.det(J))
    Jinv = np.linalg.inv(J)  # grad_x = Jinv^T grad_ref
    M2r = np.einsum("q,qa,qb->ab", wts, phi, phi)
    Gr = np.einsum("q,qam,qbn->abmn", wts, dphi, dphi)
    Cr = np.einsum("q,qe,qam->eam", wts, lam, dphi)
    Mpr = np.einsum("q,qe,qf->ef", wts, lam, lam)
    M2 = det[:, None, None] * M2r
    G = np.einsum("c,cmk,cnl,abmn->cabkl", det, Jinv, Jinv, Gr)
    C = np.einsum("c,cmk,eam->ceak", det, Jinv, Cr)
    Mp = det[:, None, None] * Mpr
    dpsi = np.einsum("cmk,em->cek", Jinv, dlam)
    Kp = (det / np.prod(np.arange(1, dim + 1)))[:, None, None] * np.einsum("cek,cfk->cef", dpsi, dpsi)
    return M2, G, C, Mp, Kp


def _vector_blocks(dim, M2, G, C):
    """Vector-P2 blocks with local dof index a*dim + c (node-major):
    Mv (mass), E (eps:eps), Dd (div div), Bt (row v, col p: int p div v)."""
    nc, nb = M2.shape[0], M2.shape[1]
    I = np.eye(dim)
    # row (b, d), col (a, c)
    Mv = np.einsum("cab,dk->cbdak", M2, I)
    lap = np.einsum("cabkk->cab", G)
    E = 0.5 * (np.einsum("cab,dk->cbdak", lap, I) + np.einsum("cabdk->cbdak", G))
    Dd = np.einsum("cabkd->cbdak", G)
    shp = (nc, nb * dim, nb * dim)
    Bt = np.einsum("cebd->cbde", C).reshape(nc, nb * dim, -1)
    return Mv.reshape(shp), E.reshape(shp), Dd.reshape(shp), Bt


def _forms(pc, prm, dim):
    """Coefficients of the elementary blocks in each matrix: a dict
    {block: [(coef, elementary name), ...]} for A, P, P_diff
    (lib/Assembler.py:66-221)."""
    phi0, phis = prm["phi0"], 1 - prm["phi0"]
    idt, ikf, dt = 1 / prm["dt"], 1 / prm["kf"], prm["dt"]
    rhos, rhof, mu_s, lmbda, mu_f, ks = prm["rhos"], prm["rhof"], prm["mu_s"], prm["lmbda"], prm["mu_f"], prm["ks"]
    a = {  # base matrix (Assembler.py:78-97)
        "ss": [(rhos * idt ** 2 * phis + phi0 ** 2 * ikf * idt, "Mv"), (2 * mu_s, "E"), (lmbda, "Dd")],
        "sf": [(-phi0 ** 2 * ikf, "Mv")],
        "sp": [(-phis, "Bt")],
        "fs": [(-phi0 ** 2 * ikf * idt, "Mv")],
        "ff": [(rhof * idt * phi0 + phi0 ** 2 * ikf, "Mv"), (2 * mu_f * phi0, "E")],
        "fp": [(-phi0, "Bt")],
        "ps": [(phis * idt, "Bq")],
        "pf": [(phi0, "Bq")],
        "pp": [(phis ** 2 * idt / ks, "Mp")],
    }
    f_rows = {k: a[k] for k in ("ff", "fp", "fs")}
    p_rows = {k: a[k] for k in ("pp", "pf", "ps")}
    cc1 = phi0 / (2 * mu_f / dim)
    cc2 = 1 / (rhof * idt / phi0 + ikf)
    beta_p = prm["betap"] * phis ** 2 / (dt * (2 * mu_s / dim + lmbda))
    mpp = phis ** 2 * idt / ks
    s_undrained = {"ss": a["ss"] + [(ks, "Dd")]}  # N div(phis u) div(phis v), N = ks / phis^2
    s_diag = {"ss": [(rhos * idt ** 2 * phis + phi0 ** 2 * ikf * (1 + prm["betas"]) * idt, "Mv"), (2 * mu_s, "E"),
                     (lmbda, "Dd")],
              "sp": [(-phis, "Bt")], "sf": [(-phi0 ** 2 * ikf, "Mv")]}
    f_diag = {"ff": [(rhof * idt * phi0 + (1 + prm["betaf"]) * phi0 ** 2 * ikf, "Mv"), (2 * mu_f * phi0, "E")],
              "fp": [(-phi0, "Bt")]}
    diff = None
    if pc == "undrained":
        P = {**s_undrained, **f_rows, **p_rows}
        diff = {}
    elif pc == "undrained 3-way":
        P = {**s_undrained, **f_rows, "pp": [(mpp + cc1, "Mp")]}
        diff = {"pp": [(mpp, "Mp"), (cc2, "Kp")]}
    elif pc == "diagonal":
        P = {**s_diag, **f_diag, "pp": [(mpp + beta_p, "Mp")], "pf": [(phi0, "Bq")]}
        diff = {}
    elif pc == "diagonal 3-way":
        P = {**s_diag, **f_diag, "pp": [(mpp + beta_p + cc1, "Mp")]}
        diff = {"pp": [(mpp + beta_p, "Mp"), (cc2, "Kp")]}
    elif pc == "diagonal 3-way-II":
        P = {**s_diag, "ff": f_diag["ff"] + [(phi0 ** 2 / (mpp + beta_p), "Dd")],
             "pp": [(mpp + beta_p, "Mp")], "pf": [(phi0, "Bq")]}
        diff = {}
    else:  # Assembler.py:214-217: P assembled from the base forms
        P = dict(a)
    Pd = None
    if "3-way" in pc:  # Poromechanics.py:21-23; a_s + a_f + a_p_diff
        Pd = {k: v for k, v in P.items() if k[0] in "sf"}
        Pd.update(diff)
    return a, P, Pd


# ------------------------------------------------------------- assembly --
def _numbering(dim, cell_nodes, nv, nnodes, ordering):
    """Global dof numbers of (node, comp) for u_s and v_f, and of vertex p."""
    nc, nb = cell_nodes.shape
    r = np.repeat(cell_nodes, nb, 1).ravel()
    c = np.tile(cell_nodes, (1, nb)).ravel()
    g = sp.csr_matrix((np.ones(r.size, dtype=np.int8), (r, c)), shape=(nnodes, nnodes))
    order = np.asarray(reverse_cuthill_mckee(g, symmetric_mode=True), dtype=np.int64)
    rank = np.empty(nnodes, dtype=np.int64)
    rank[order] = np.arange(nnodes)
    ns = dim * nnodes
    if ordering == "field-major":
        us = rank[:, None] * dim + np.arange(dim)
        vf = ns + us
        vrank = np.argsort(np.argsort(rank[:nv], kind="stable"), kind="stable")
        p = 2 * ns + vrank
    elif ordering == "interleaved":
        per = 2 * dim + (order < nv)  # dofs per node in RCM order
        start = np.concatenate([[0], np.cumsum(per)[:-1]])
        s_node = np.empty(nnodes, dtype=np.int64)
        s_node[order] = start
        us = s_node[:, None] + np.arange(dim)
        vf = s_node[:, None] + dim + np.arange(dim)
        p = s_node[:nv] + 2 * dim
    else:
        raise ValueError(f"unknown ordering {ordering!r}")
    return us, vf, p


def _dirichlet(M, rows):
    """dolfin DirichletBC.apply(A): zero the rows, unit diagonal."""
    M = M.tocsr(copy=True)
    for r in rows:
        lo, hi = M.indptr[r], M.indptr[r + 1]
        M.data[lo:hi] = 0.0
        d = lo + np.searchsorted(M.indices[lo:hi], r)
        assert d < hi and M.indices[d] == r
        M.data[d] = 1.0
    return M


def assemble_forms(dim, xcells, cells, cell_nodes, nv, nnodes, pc_type, prm, ordering):
    """A, P, P_diff (None unless 3-way) of ``pc_type`` on a simplicial mesh
    (physical vertex coordinates per cell ``xcells``; P2 nodes ``cell_nodes``:
    the cell's vertices, then its edges in ``itertools.combinations`` order)
    and the dof numbers (us, vf, p) -- shared by the swelling and footing
    assemblers (lib/Assembler.py:66-221)."""
    M2, G, C, Mp, Kp = _element_blocks(dim, xcells)
    Mv, E, Dd, Bt = _vector_blocks(dim, M2, G, C)
    elem = {"Mv": Mv, "E": E, "Dd": Dd, "Bt": Bt, "Bq": np.transpose(Bt, (0, 2, 1)), "Mp": Mp, "Kp": Kp}

    us, vf, p = _numbering(dim, cell_nodes, nv, nnodes, ordering)
    nc, nb = cell_nodes.shape
    ldofs = {"s": us[cell_nodes].reshape(nc, nb * dim), "f": vf[cell_nodes].reshape(nc, nb * dim),
             "p": p[cells]}
    loc = np.concatenate([ldofs["s"], ldofs["f"], ldofs["p"]], 1)
    nl = loc.shape[1]
    n = 2 * dim * nnodes + nv
    rows = np.repeat(loc, nl, 1).ravel()
    cols = np.tile(loc, (1, nl)).ravel()
    offs = {"s": 0, "f": nb * dim, "p": 2 * nb * dim}
    size = {"s": nb * dim, "f": nb * dim, "p": dim + 1}

    def build(form):
        K = np.zeros((nc, nl, nl))
        for blk, terms in form.items():
            r0, c0 = offs[blk[0]], offs[blk[1]]
            for coef, name in terms:
                K[:, r0:r0 + size[blk[0]], c0:c0 + size[blk[1]]] += coef * elem[name]
        M = sp.coo_matrix((K.ravel(), (rows, cols)), shape=(n, n)).tocsr()
        M.sum_duplicates()
        M.sort_indices()
        return M

    fa, fp_, fd = _forms(pc_type, prm, dim)
    A, P = build(fa), build(fp_)
    Pd = build(fd) if fd is not None else None
    return A, P, Pd, (us, vf, p)


def assemble_swelling(dim: int, N: int, pc_type: str = "diagonal", params: dict | None = None,
                      ordering: str = "field-major", t: float | None = None) -> SwellingSystem:
    """The swelling (dim 2: swelling.py) / swelling-3d (dim 3) system at the
    first time step: A, P, P_diff (None unless ``"3-way" in pc_type``), b,
    index sets and pressure-BC positions, as the reference hands them to
    ``Preconditioner`` / ``Solver`` (lib/Poromechanics.py:58-98)."""
    if dim not in (2, 3):
        raise ValueError("dim must be 2 or 3")
    prm = dict(SWELLING_2D if dim == 2 else SWELLING_3D, **(params or {}))
    t = prm["dt"] if t is None else t
    coords, cells, pairs, cell_nodes, node2x, nv = _p2_nodes(dim, N)
    nnodes = node2x.shape[0]
    h = SIDE_LENGTH / N
    A, P, Pd, (us, vf, p) = assemble_forms(dim, coords[cells].astype(np.float64) * h, cells, cell_nodes, nv, nnodes,
                                           pc_type, prm, ordering)
    n = A.shape[0]

    # ---- right-hand side: surface tractions at time t (Assembler.py:235-269)
    cs = -1e3 * 0.9 * (1 - np.exp(-t ** 2 / 0.25))
    cf = -1e3 * 0.1 * (1 - np.exp(-t ** 2 / 0.25))
    if dim == 2:  # LEFT x-, RIGHT x+, TOP y+, BOTTOM y- ; sides as (axis, at_max)
        neu_s, neu_f = [(1, True), (0, True)], [(0, False)]
        bc_s = [(0, (0, False)), (1, (1, False))]
        bc_f = [(1, True), (1, False)]
        bc_p = [(0, False), (1, True), (0, True)]
    else:  # swelling-3d.py:21-22,95-106
        neu_s, neu_f = [(0, True), (1, True), (2, True)], [(0, False), (1, False)]
        bc_s = [(0, (0, False)), (1, (1, False)), (2, (2, False))]
        bc_f = [(2, False), (2, True)]
        bc_p = [(0, False), (0, True), (1, False), (1, True), (2, True)]
    b = np.zeros(n)
    fac_k = dim - 1
    w_vert = 4.0 / ((fac_k + 1) * (fac_k + 2)) - 1.0 / (fac_k + 1)
    w_edge = 4.0 / ((fac_k + 1) * (fac_k + 2))
    area = h ** fac_k / np.prod(np.arange(1, fac_k + 1))
    for c, sides, field in ((cs, neu_s, us), (cf, neu_f, vf)):
        for axis, at_max in sides:
            val = N if at_max else 0
            normal = 1.0 if at_max else -1.0
            for omit in range(dim + 1):  # facet = cell minus vertex `omit`
                lv = [i for i in range(dim + 1) if i != omit]
                on = np.all(coords[cells[:, lv], axis] == val, 1)
                if not on.any():
                    continue
                for i in lv:
                    np.add.at(b, field[cells[on, i], axis], c * normal * w_vert * area)
                for e, (i, j) in enumerate(pairs):
                    if i != omit and j != omit:
                        np.add.at(b, field[cell_nodes[on, dim + 1 + e], axis], c * normal * w_edge * area)

    def nodes_on(axis, at_max):
        return np.nonzero(node2x[:, axis] == (2 * N if at_max else 0))[0]

    bc_rows = [us[nodes_on(*side), comp] for comp, side in bc_s]
    bc_rows += [vf[nodes_on(*side)].ravel() for side in bc_f]
    bc_rows = np.unique(np.concatenate(bc_rows))
    p_rows = np.unique(np.concatenate([p[nodes_on(*side)[nodes_on(*side) < nv]] for side in bc_p]))
    A, P = _dirichlet(A, bc_rows), _dirichlet(P, bc_rows)
    b[bc_rows] = 0.0
    if Pd is not None:
        Pd = _dirichlet(_dirichlet(Pd, bc_rows), p_rows)

    is_s, is_f, is_p = (np.sort(x.ravel()).astype(np.int32) for x in (us, vf, p))
    bcs_sub = np.searchsorted(is_p, p_rows).astype(np.int32)
    return SwellingSystem(A, P, Pd, b, is_s, is_f, is_p, bcs_sub, dim, N)
