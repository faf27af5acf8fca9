"""ExpDiskGeometry (SKIRTcore/ExpDiskGeometry.cpp, SepAxGeometry::generatePosition,
SpecialFunctions::LambertW1) in the host model and the oracle.

The disk_oct, disk_cart, bulge_oct, sersic_cart and point_oct reference fixtures pin these geometries
(tests/test_oracle_golden.py); these tests pin the restatement to its own defining properties:
the density formula and its normalization (setupSelfBefore's rho0 makes the density integrate to 1),
and the random positions (randomR by LambertW1 inversion, randomz, the truncations) distributed as
that density. The GPU engine then matches the oracle on the same streams (tests/test_gpu_geometries.py).
"""
import math

import numpy as np
import pytest

import oracle_lib as O
import tree_models as T

PC = 3.08567758e16  # the parsec of the host units (host/units.hpp, Units.cpp of the reference)


def disk_pdf_R(R, hR, Rmin, Rmax):
    """Radial probability density of an exponential disk, R exp(-R/hR) on [Rmin, Rmax)."""
    f = R * np.exp(-R / hR)
    grid = np.linspace(Rmin, Rmax if Rmax > 0 else 40 * hR, 200001)
    norm = np.trapezoid(grid * np.exp(-grid / hR), grid)
    return f / norm


@pytest.mark.parametrize("comp_geom", ["star", "dust"])
def test_exp_disk_positions_follow_the_density(tmp_path, comp_geom):
    # a model whose stellar component carries the geometry under test
    base, star, dust = T.GEOMETRIES["disk_cart"]
    geom = star if comp_geom == "star" else dust
    T.GEOMETRIES["_probe"] = (base, geom, dust)
    try:
        path = T.write_geometry("_probe", str(tmp_path))
    finally:
        del T.GEOMETRIES["_probe"]
    n = 200000
    pos, dens = O.star_positions(path, 0, n, seed=12345)
    R = np.hypot(pos[:, 0], pos[:, 1])
    z = pos[:, 2]
    if comp_geom == "star":
        hR, hz, Rmax, zmax, Rmin = 120 * PC, 25 * PC, 0.0, 0.0, 0.0
    else:
        hR, hz, Rmax, zmax, Rmin = 150 * PC, 40 * PC, 450 * PC, 300 * PC, 20 * PC
    # truncations hold exactly
    assert np.all(R > Rmin)
    if Rmax > 0:
        assert np.all(R < Rmax)
    if zmax > 0:
        assert np.all(np.abs(z) < zmax)
    # every sampled point has positive density, with the separable form rho0 exp(-R/hR) exp(-|z|/hz)
    assert np.all(dens > 0)
    rho0 = dens * np.exp(R / hR) * np.exp(np.abs(z) / hz)
    np.testing.assert_allclose(rho0, rho0[0], rtol=1e-12)
    # normalization: rho0 = 1 / (int R dR * 2 pi * int dz)  (ExpDiskGeometry::setupSelfBefore)
    intz = -2 * hz * math.expm1(-zmax / hz) if zmax > 0 else 2 * hz
    tmin = math.exp(-Rmin / hR) * (1 + Rmin / hR) if Rmin > 0 else 1.0
    tmax = math.exp(-Rmax / hR) * (1 + Rmax / hR) if Rmax > 0 else 0.0
    np.testing.assert_allclose(rho0[0], 1.0 / (hR * hR * (tmin - tmax) * 2 * math.pi * intz), rtol=1e-9)
    # azimuths uniform, heights Laplace with scale hz (truncated), radii R exp(-R/hR)
    phi = np.arctan2(pos[:, 1], pos[:, 0])
    assert abs(np.mean(np.cos(phi))) < 0.01 and abs(np.mean(np.sin(phi))) < 0.01
    az = np.abs(z)
    zc = zmax if zmax > 0 else np.inf
    mean_az = hz - (zc * math.exp(-zc / hz) / -math.expm1(-zc / hz) if zmax > 0 else 0.0)
    assert abs(az.mean() - mean_az) < 5 * az.std() / math.sqrt(n)
    edges = np.linspace(max(Rmin, 1e-3 * hR), Rmax if Rmax > 0 else 8 * hR, 41)
    counts, _ = np.histogram(R, bins=edges)
    mids = 0.5 * (edges[1:] + edges[:-1])
    expected = disk_pdf_R(mids, hR, Rmin, Rmax) * np.diff(edges) * n
    ok = expected > 100
    chi = (counts[ok] - expected[ok]) / np.sqrt(expected[ok])
    assert np.all(np.abs(chi) < 6) and np.mean(chi ** 2) < 2.0, chi


@pytest.mark.parametrize("name", ["disk_cart", "disk_oct", "bulge_oct", "sersic_cart", "point_oct", "point_cart"])
def test_geometry_models_run_deterministically(tmp_path, name):
    """The oracle's MT mode (the reference's -t 1 draw order) runs the disk models; two runs agree bit
    for bit and the tallies are positive and finite."""
    path = T.write_geometry(name, str(tmp_path))
    a = O.run(path, rng=O.RNG_MT, threads=1, packages=300)
    b = O.run(path, rng=O.RNG_MT, threads=1, packages=300)
    assert a.packets == b.packets > 0
    np.testing.assert_array_equal(a.labs, b.labs)
    assert np.isfinite(a.labs).all() and a.labs.sum() > 0
    np.testing.assert_array_equal(a.seds[0], b.seds[0])


@pytest.mark.parametrize("geom,n,reff_pc", [("SERSIC4", 4.0, 60.0), ("SERSIC1", 1.5, 120.0)])
def test_sersic_positions_have_the_effective_radius(tmp_path, geom, n, reff_pc):
    """SersicGeometry: the deprojected profile (SersicFunction's tables) sampled by inverse mass and an
    isotropic direction puts half of the projected light inside reff -- the defining property of the
    effective radius, independent of the tables' construction. Also rho = rho0 S(r/reff) > 0."""
    base = "pan_cart16"
    T.GEOMETRIES["_probe"] = (base, getattr(T, geom), T.DUST_DISK)
    try:
        path = T.write_geometry("_probe", str(tmp_path))
    finally:
        del T.GEOMETRIES["_probe"]
    N = 400000
    pos, dens = O.star_positions(path, 0, N, seed=777)
    reff = reff_pc * PC
    Rproj = np.hypot(pos[:, 0], pos[:, 1])
    frac = np.mean(Rproj < reff)
    assert abs(frac - 0.5) < 0.005, frac
    assert np.all(dens > 0)
    r = np.linalg.norm(pos, axis=1)
    # isotropy and a density decreasing with radius
    assert abs(np.mean(pos[:, 2] / r)) < 0.01
    order = np.argsort(r)
    assert np.all(np.diff(dens[order][:: N // 50]) <= 0)


def test_point_geometry_positions_are_the_origin(tmp_path):
    """PointGeometry (SKIRTcore/PointGeometry.cpp): generatePosition returns the origin without random
    draws, the density is infinite there and zero elsewhere."""
    path = T.write_geometry("point_oct", str(tmp_path))
    pos, dens = O.star_positions(path, 0, 1000, seed=5)
    assert np.all(pos == 0.0)
    assert np.all(np.isinf(dens))


def test_point_geometry_is_refused_for_dust(tmp_path):
    T.GEOMETRIES["_pdust"] = ("pan_oct", T.STAR_DISK, T.POINT)
    try:
        path = T.write_geometry("_pdust", str(tmp_path))
    finally:
        del T.GEOMETRIES["_pdust"]
    with pytest.raises(RuntimeError, match="PointGeometry"):
        O.run(path, rng=O.RNG_MT, threads=1, packages=10)
