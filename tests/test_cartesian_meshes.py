"""Cartesian dust grid meshes (CartesianDustGrid.cpp:34-36 with LinMesh / PowMesh / SymPowMesh, i.e.
NR::lingrid / NR::powgrid / NR::sympowgrid, Fundamentals/NR.hpp:171-261): the borders the host builds
are the reference's formulas evaluated in the same order, read back through the oracle's
DustGrid::path along each axis. No reference fixture uses these meshes, so beyond these formulas the
power-law meshes are pinned against the reference by the cart_pow and cart_odd fixtures (the GPU engine matches the oracle
on them, tests/test_gpu_cartesian.py)."""
import math

import numpy as np
import pytest

import oracle_lib as O
import tree_models as T


def lingrid(n):
    dx = (1.0 - 0.0) / n
    return [0.0 + i * dx for i in range(n + 1)]


def powgrid(n, ratio):
    if n <= 1 or abs(ratio - 1.0) < 1e-3:
        return lingrid(n)
    q = math.pow(ratio, 1.0 / (n - 1))
    qn = math.pow(q, n)
    return [0.0 + (1.0 - math.pow(q, i)) / (1.0 - qn) * (1.0 - 0.0) for i in range(n + 1)]


def sympowgrid(n, ratio):
    if n <= 2 or abs(ratio - 1.0) < 1e-3:
        return lingrid(n)
    xv = [0.0] * (n + 1)
    xc = 0.5 * (0.0 + 1.0)
    if n % 2 == 0:
        M = n // 2
        q = math.pow(ratio, 1.0 / (M - 1.0))
        qM = math.pow(q, M)
        xv[M] = xc
        for i in range(1, M + 1):
            d = (1.0 - math.pow(q, i)) / (1.0 - qM) * 0.5 * (1.0 - 0.0)
            xv[M + i] = xc + d
            xv[M - i] = xc - d
    else:
        M = (n + 1) // 2
        q = math.pow(ratio, 1.0 / (M - 1.0))
        qM = math.pow(q, M)
        for i in range(1, M + 1):
            d = (0.5 + 0.5 * q - math.pow(q, i)) / (0.5 + 0.5 * q - qM) * 0.5 * (1.0 - 0.0)
            xv[M - 1 + i] = xc + d
            xv[M - i] = xc - d
    return xv


def axis_borders(path, axis):
    """The cell borders the grid's path crosses along `axis` (a ray along that axis through the grid)."""
    ray = np.zeros((1, 6))
    ray[0, :3] = 1e15  # off the other axes' borders (all meshes are symmetric about 0 or not, any point)
    ray[0, axis] = -1e30
    ray[0, 3 + axis] = 1.0
    (boxes, ds), = O.grid_paths(path, ray)[0]
    boxes = boxes[~np.isnan(boxes[:, 0])]
    return np.concatenate([boxes[:, axis], boxes[-1:, 3 + axis]])


@pytest.mark.parametrize("name,meshes", [
    ("cart_odd", [lingrid(7), lingrid(5), lingrid(9)]),
    ("cart_pow", [powgrid(12, 4.0), sympowgrid(9, 3.0), sympowgrid(10, 0.2)]),
])
def test_cartesian_mesh_borders_follow_the_reference_formulas(tmp_path, name, meshes):
    path = T.write(name, str(tmp_path))
    for axis, tv in enumerate(meshes):
        b = axis_borders(path, axis)
        assert len(b) == len(tv)
        lo, hi = b[0], b[-1]
        expected = np.array([t * (hi - lo) + lo for t in tv])
        np.testing.assert_array_equal(b, expected)
