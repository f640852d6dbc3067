"""The footing assembler (lib/fe_footing.py; footing.py + lib/MeshCreation.py:53-77):
mesh geometry of the twice locally refined square, the traction load and the
footing BCs, and the committed footing fixtures (host only, no GPU).

Nothing here is pinned against dolfin (absent): the mesh by its geometry
(area, conformity, refined cell sizes), the loads and BCs by closed forms."""
import json
import os

import numpy as np
import pytest

from lib import fe_footing as FF

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "footing")


def _areas(c, cells):
    x = c[cells]
    return 0.5 * np.abs((x[:, 1, 0] - x[:, 0, 0]) * (x[:, 2, 1] - x[:, 0, 1])
                        - (x[:, 2, 0] - x[:, 0, 0]) * (x[:, 1, 1] - x[:, 0, 1]))


@pytest.mark.parametrize("N", [4, 8, 16])
def test_mesh_is_conforming_and_covers_the_square(N):
    c, cells = FF.footing_mesh(N)
    a = _areas(c, cells)
    assert np.isclose(a.sum(), FF.LENGTH ** 2, rtol=1e-14)
    assert a.min() > 0
    # a hanging node would leave an interior edge with one cell: the boundary
    # edges must be exactly the square's perimeter
    bf, _ = FF.boundary_facets(cells)
    xa, xb = c[bf[:, 0]], c[bf[:, 1]]
    on_side = ((xa[:, 0] == xb[:, 0]) & np.isin(xa[:, 0], [0, FF.LENGTH])) | \
              ((xa[:, 1] == xb[:, 1]) & np.isin(xa[:, 1], [0, FF.LENGTH]))
    assert on_side.all()
    assert np.isclose(np.linalg.norm(xb - xa, axis=1).sum(), 4 * FF.LENGTH, rtol=1e-14)
    # every interior edge is shared by exactly two cells
    uniq, c2e = FF._edges(cells)
    assert np.bincount(c2e.ravel()).max() == 2


def test_refinement_region_and_cell_sizes():
    """Cells of the base grid have area h^2/2; inside the marked region (top
    third, x in (L/8, 7L/8)) two refinements quarter them twice: h^2/32;
    outside the region and its one-cell transition band cells are untouched."""
    N = 16
    h = FF.LENGTH / N
    c, cells = FF.footing_mesh(N)
    a = _areas(c, cells)
    cen = c[cells].mean(1)
    assert set(np.unique(np.round(a / h ** 2, 12))) <= {0.5, 0.25, 0.125, 0.0625, 0.03125}
    deep = (cen[:, 1] > 2 * FF.LENGTH / 3 + 2 * h) & (cen[:, 0] > FF.LENGTH / 8 + 2 * h) & \
           (cen[:, 0] < 7 * FF.LENGTH / 8 - 2 * h)
    assert np.allclose(a[deep], h ** 2 / 32)
    far = (cen[:, 1] < 2 * FF.LENGTH / 3 - 2 * h) | (cen[:, 0] < FF.LENGTH / 8 - 2 * h) | \
          (cen[:, 0] > 7 * FF.LENGTH / 8 + 2 * h)
    assert np.allclose(a[far], h ** 2 / 2)


def test_plaza_single_triangle_and_neighbour_closure():
    """Two right triangles sharing the hypotenuse: marking one refines it into
    four (all edges marked, edge ratio sqrt(2)/2 -> red) and the neighbour
    bisects its longest edge (the shared hypotenuse) to stay conforming."""
    c = np.array([[0., 0.], [1., 0.], [1., 1.], [0., 1.]])
    cells = np.array([[0, 1, 2], [0, 2, 3]])
    c2, cells2 = FF.plaza_refine(c, cells, np.array([True, False]))
    a = _areas(c2, cells2)
    assert np.isclose(a.sum(), 1.0)
    assert cells2.shape[0] == 4 + 2 and c2.shape[0] == 4 + 3
    bf, _ = FF.boundary_facets(cells2)
    assert np.isclose(np.linalg.norm(c2[bf[:, 1]] - c2[bf[:, 0]], axis=1).sum(), 4.0)


def test_dof_count_estimate_at_configs2_size():
    """the footing mesh refined twice near the top has about
    4-5x the base grid's DoF (exact count needs dolfin); N = 128 here."""
    N = 128
    c, cells = FF.footing_mesh(N)
    nv, ne = c.shape[0], FF._edges(cells)[0].shape[0]
    n = 4 * (nv + ne) + nv
    base = 4 * (2 * N + 1) ** 2 + (N + 1) ** 2
    assert base == 280_837
    assert 4.0 < n / base < 5.0


@pytest.mark.parametrize("N", [8, 12])
def test_traction_load_and_bcs(N):
    s = FF.assemble_footing(N, "undrained 3-way")
    n = s.A.shape[0]
    h_top = FF.LENGTH / N / 4  # top edges lie inside the twice refined region
    # total load = integral of the P1 interpolant of fs_sur over the top: the
    # step |x - 32| < 16 loses one top edge (half at each end) to interpolation
    assert np.isclose(s.b.sum(), -1e4 * (FF.LENGTH / 2 - h_top), rtol=1e-13)
    nz = np.nonzero(s.b)[0]
    assert np.isin(nz, s.is_s).all()
    # Dirichlet rows: unit rows in A and P, zero rhs
    A = s.A.tocsr()
    d = A.diagonal()
    rows_unit = np.nonzero((np.diff(A.indptr) > 0) & (d == 1.0) & (np.abs(A).sum(1).A1 == 1.0))[0]
    # solid bottom: 2 comps x (2N*... P2 nodes on y = 0: 2N + 1), fluid foot: 2 comps x foot P2 nodes
    n_bottom = 2 * (2 * N + 1)
    # strict |x - 32| < 16 on every vertex: the facets between x = 16 + h and 48 - h,
    # 32/h - 2 of them, 2 (32/h - 2) + 1 P2 nodes
    foot_nodes = 2 * (int(round((FF.LENGTH / 2) / h_top)) - 2) + 1
    assert rows_unit.size == n_bottom + 2 * foot_nodes
    assert np.all(s.b[rows_unit] == 0.0)
    # pressure BCs (P_diff only): every boundary vertex not on the foot
    Pd = s.P_diff.tocsr()
    p_rows = s.is_p[s.bcs_sub_pressure]
    assert np.all(Pd.diagonal()[p_rows] == 1.0)
    assert np.all(np.abs(Pd[p_rows]).sum(1).A1 == 1.0)
    n_bverts = 4 * N + (N // 2) * (4 - 1) * 2  # perimeter vertices: 3 coarse sides + the top (refined 4x in x in (8,56))
    assert p_rows.size < n_bverts
    assert s.A.shape == (n, n) and s.P.shape == (n, n)


@pytest.mark.parametrize("name", ["footing_N8_undrained_exact", "footing_N8_undrained_inexact_ilu",
                                  "footing_N8_3way_exact"])
def test_footing_golden_fixture(name):
    """Assembler (checksums, sizes) and oracle (its, reason, history, x)
    against the committed fixture (tests/golden/make_golden_footing.py)."""
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    import make_golden_footing as G
    z = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    s = FF.assemble_footing(meta["N"], meta["pc"])
    assert tuple(s.dims) == tuple(z["dims"]) and s.A.nnz == int(z["nnz"])
    assert np.array_equal(np.asarray(s.bcs_sub_pressure), z["bcs_sub_pressure"])
    assert np.allclose(G.checksums(s), z["checksums"], rtol=1e-12, atol=0)
    s2, params, db, o, x = G.run_case(name)
    assert o.its == int(z["its"]) and o.reason == int(z["reason"])
    assert np.allclose(np.asarray(o.history), z["history"], rtol=1e-8, atol=0)
    assert np.linalg.norm(x - z["x"]) <= 1e-8 * np.linalg.norm(z["x"])
