"""Tree dust grids beyond the pinned octree fixture: the k-d tree (BinTreeDustGrid), barycentric
subdivision and the TopDown search, on the CPU oracle (tests/tree_models.py explains the pinning).

A full k-d tree of level 3L splits x, y and z at the box centres in turn (BinTreeNode.cpp:38-66, level
% 3), so its leaves are exactly the leaves of the full octree of level L; the reference's path through
both therefore crosses the same boxes over the same distances. The octree walk is pinned bit for bit
to the reference (tests/test_oracle_golden.py), so equal paths pin the k-d tree's construction, its
neighbour lists (BinTreeNode::addneighbors) and its descent (BinTreeNode::child).
"""
import numpy as np
import pytest

import oracle_lib as O
import tree_models as T

PC = 3.0856775807e16  # m


def rays(n, seed):
    rng = np.random.default_rng(seed)
    pos = rng.uniform(-650, 650, (n, 3)) * PC  # inside the grid and around it
    pos[: n // 4] = rng.uniform(-30, 30, (n // 4, 3)) * PC  # near the centre, where the cells are small
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[:8] = [[1, 0, 0], [0, -1, 0], [0, 0, 1], [-1, 0, 0], [0.6, 0.8, 0], [0, 0.6, -0.8], [0.8, 0, 0.6], [0, 1, 0]]
    return np.hstack([pos, d])


@pytest.mark.parametrize("bin_name", ["bin_full", "bin_full_td"])
def test_full_kd_tree_paths_equal_full_octree_paths(tmp_path, bin_name):
    r = rays(400, 7)
    oct_paths, n_oct = O.grid_paths(T.write("oct_full", str(tmp_path)), r)
    bin_paths, n_bin = O.grid_paths(T.write(bin_name, str(tmp_path)), r)
    assert n_oct == n_bin == 16 ** 3
    crossed = 0
    for (bo, do), (bb, db) in zip(oct_paths, bin_paths):
        assert len(do) == len(db)
        np.testing.assert_array_equal(bo, bb)  # the same cell boxes (NaN before the grid)
        np.testing.assert_array_equal(do, db)  # over exactly the same distances
        crossed += len(do)
    assert crossed > 400 * 10


def test_kd_tree_search_methods_agree(tmp_path):
    """Neighbor and TopDown searches walk the same adaptive k-d tree to the same cells."""
    r = rays(300, 11)
    a, na = O.grid_paths(T.write("bin_pan", str(tmp_path)), r)
    b, nb = O.grid_paths(T.write("bin_pan_td", str(tmp_path)), r)
    assert na == nb
    for (ba, da), (bb, db) in zip(a, b):
        np.testing.assert_array_equal(ba, bb)
        np.testing.assert_array_equal(da, db)


@pytest.mark.parametrize("name", ["bin_pan", "bin_bary", "oct_bary"])
def test_tree_paths_tile_the_grid(tmp_path, name):
    """Every path through an adaptive tree is a chain of cell boxes: consecutive segments are
    contiguous along the ray, every segment lies inside its box, and a ray through the whole grid
    covers its full chord."""
    r = rays(200, 3)
    paths, ncells = O.grid_paths(T.write(name, str(tmp_path)), r)
    assert ncells > 1000
    lo, hi = -500 * PC, 500 * PC
    for q, (boxes, ds) in zip(r, paths):
        if not len(ds):
            continue
        inside = ~np.isnan(boxes[:, 0])
        assert inside.any()
        assert (boxes[inside, :3] < boxes[inside, 3:]).all()
        assert (boxes[inside, :3] >= lo).all() and (boxes[inside, 3:] <= hi).all()
        s = np.cumsum(ds)
        p0, k = q[:3], q[3:]
        # the midpoint of every segment inside the grid lies in (or on the faces of) its box
        mid = p0[None, :] + k[None, :] * (s - 0.5 * ds)[:, None]
        tol = 1e-9 * (hi - lo)
        b = boxes[inside]
        assert (mid[inside] >= b[:, :3] - tol).all() and (mid[inside] <= b[:, 3:] + tol).all()
        # the path ends on the grid boundary
        end = p0 + k * s[-1]
        assert np.isclose(np.abs(end).max(), hi, rtol=1e-6)


def test_barycentric_trees_split_off_centre(tmp_path):
    """BaryOctTreeNode / BaryBinTreeNode split at the sampled barycentre (octree) or along the axis
    whose wall lies nearest to it (k-d tree): off-centre boxes for the octree, and for the k-d tree
    boxes whose aspect ratios differ from the alternating tree's."""
    r = rays(100, 5)
    ob, _ = O.grid_paths(T.write("oct_bary", str(tmp_path)), r)
    boxes = np.vstack([b for b, _ in ob if len(b)])
    boxes = boxes[~np.isnan(boxes[:, 0])]
    w = boxes[:, 3:] - boxes[:, :3]
    # centre splits give widths 1000 pc / 2^n; barycentric ones do not
    lev = np.log2(1000 * PC / w)
    assert (np.abs(lev - np.round(lev)) > 1e-6).any()
    bb, _ = O.grid_paths(T.write("bin_bary", str(tmp_path)), r)
    boxes = np.vstack([b for b, _ in bb if len(b)])
    boxes = boxes[~np.isnan(boxes[:, 0])]
    w = boxes[:, 3:] - boxes[:, :3]
    lev = np.log2(1000 * PC / w)
    np.testing.assert_allclose(lev, np.round(lev), atol=1e-9)  # always halves
    per_axis = np.round(lev).astype(int)
    alternating = (per_axis[:, 0] >= per_axis[:, 1]) & (per_axis[:, 1] >= per_axis[:, 2]) & \
                  (per_axis[:, 0] - per_axis[:, 2] <= 1)
    assert not alternating.all()


@pytest.mark.parametrize("name", ["bin_pan", "bin_bary", "oct_bary", "oct_pan_td"])
def test_tree_variants_run_in_both_rng_modes(tmp_path, name):
    path = T.write(name, str(tmp_path))
    mt = O.run(path, rng=O.RNG_MT, packages=3000)
    ph = O.run(path, rng=O.RNG_PHILOX, threads=4, packages=3000)
    assert mt.packets == ph.packets > 0
    for res in (mt, ph):
        assert np.isfinite(res.labs).all() and res.labs.sum() > 0
    # the two streams estimate the same absorbed luminosity
    np.testing.assert_allclose(mt.labs.sum(), ph.labs.sum(), rtol=0.1)


@pytest.mark.parametrize("nb,bk", [("pan_oct", "oct_pan_bk"), ("oct_bary", "oct_bary_bk")])
def test_bookkeeping_search_crosses_the_neighbor_search_cells(tmp_path, nb, bk):
    """The Bookkeeping search (TreeDustGrid.cpp:523-659) puts the position on each crossed wall instead of
    eps beyond it, so its segments differ from the Neighbor search's by about eps; it crosses the same
    cells in the same order (apart from rays through a cell edge or corner, where the two searches may
    legitimately pick different cells) and covers the same chord."""
    import os
    r = rays(300, 13)
    src = os.path.join(T.GOLD, "pan_oct.ski") if nb == "pan_oct" else T.write(nb, str(tmp_path))
    a, na = O.grid_paths(src, r)
    b, nb_ = O.grid_paths(T.write(bk, str(tmp_path)), r)
    assert na == nb_
    same = 0
    eps = 1e-12 * np.sqrt(3) * 1000 * PC
    for (ba, da), (bb, db) in zip(a, b):
        if len(da) == len(db) and np.array_equal(ba, bb, equal_nan=True):
            same += 1
            np.testing.assert_allclose(da, db, rtol=0, atol=4 * eps)
        if len(da):
            np.testing.assert_allclose(da.sum(), db.sum(), rtol=1e-9)
    assert same >= 0.99 * len(r)
