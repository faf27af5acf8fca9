"""The setup on the device (skirt_sim_load_ex / Simulation(setup_device=0)) against the host setup, which is
bit-identical to the reference (tests/test_oracle_golden.py): the density sampling (skirt_mcrt_sample_density:
the same random words, the same tree, and cell densities equal to an ulp of the device's exp/pow/log10,
relative tolerance 1e-13) and a Voronoi grid's cells (skirt_mcrt_voronoi_cells: the host tessellation bit for
bit). Reference: DustSystem::setupSelfAfter (DustSystem.cpp:152-178), TreeNodeSampleDensityCalculator
(TreeDustGrid.cpp:174-222), VoronoiMesh (VoronoiMesh.cpp:310-376, Voro++)."""
import ctypes
import os
import time

import numpy as np
import pytest

import skirt_amd as S
import tree_models as T

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKI = os.path.join(REPO, "tests", "golden", "ski")


def _compare(path):
    host = S.Simulation(path)
    dev = S.Simulation(path, setup_device=0)
    assert dev.info.ncells == host.info.ncells
    assert dev.info.nnodes == host.info.nnodes
    rh, rd = host.density(), dev.density()
    assert rh.shape == rd.shape
    np.testing.assert_allclose(rd, rh, rtol=1e-13, atol=0)
    return host, dev


@pytest.mark.parametrize("name", ["pan_oct.ski", "pan_cart16.ski", "oligo_2comp.ski", "pan_oct_sa.ski"])
def test_device_setup_matches_host(name):
    _compare(os.path.join(SKI, name))


@pytest.mark.parametrize("name", ["disk_cart", "disk_oct", "bulge_oct", "sersic_cart"])
def test_device_setup_geometries(tmp_path, name):
    _compare(T.write_geometry(name, str(tmp_path)))


def test_device_setup_c3_tree():
    """The full C3 octree (711k nodes): the same subdivision, densities to an ulp; reports both setup times."""
    path = os.path.join(REPO, "benchmarks", "c3_oct128.ski")
    t0 = time.time()
    host = S.Simulation(path)
    t1 = time.time()
    dev = S.Simulation(path, setup_device=0)
    t2 = time.time()
    print("C3 setup: host %.2f s, device density sampling %.2f s" % (t1 - t0, t2 - t1))
    assert dev.info.nnodes == host.info.nnodes and dev.info.ncells == host.info.ncells
    np.testing.assert_allclose(dev.density(), host.density(), rtol=1e-13, atol=0)


def test_device_setup_then_photon_phase_matches_host_setup():
    """A simulation set up with device sampling runs its photon phase like one set up on the host (the
    same tree; densities equal to an ulp, so the tallies agree to the same-stream tolerance)."""
    from parity import STELLAR_OUTLIERS, assert_parity
    path = os.path.join(SKI, "pan_oct.ski")
    out = []
    for dev in (None, 0):
        sim = S.Simulation(path, packages=2000, setup_device=dev)
        sim.attach(0)
        sim.run_stellar()
        sim.fetch()
        out.append((sim.labs(), sim.instrument(0)[1]))
    (la, sa), (lb, sb) = out
    np.testing.assert_allclose(lb.sum(axis=0), la.sum(axis=0), rtol=1e-9)
    assert_parity(lb, la, 1e-9, STELLAR_OUTLIERS, "labs (device setup)")
    np.testing.assert_allclose(sb, sa, rtol=1e-9, atol=1e-300)


@pytest.mark.parametrize("name", ["vor_oligo.ski", "vor_pan.ski"])
def test_device_setup_voronoi_models(name):
    """Voronoi models set up on the device (cells and density sampling): the same cells (the densities are
    sampled at positions drawn in each cell's bounding box and kept by isPointClosestTo, so any difference
    in a box or a neighbour list would move them), densities to an ulp."""
    _compare(os.path.join(SKI, name))


def test_device_setup_c4_voronoi():
    """C4's 1e5-site tessellation set up on the device: the same cells and densities; reports both times."""
    path = os.path.join(REPO, "benchmarks", "c4_vor1e5.ski")
    t0 = time.time()
    host = S.Simulation(path)
    t1 = time.time()
    dev = S.Simulation(path, setup_device=0)
    t2 = time.time()
    print("C4 setup: host %.2f s, device %.2f s" % (t1 - t0, t2 - t1))
    assert dev.info.ncells == host.info.ncells == 100000
    np.testing.assert_allclose(dev.density(), host.density(), rtol=1e-13, atol=0)


class _GridDesc(ctypes.Structure):  # SkirtGridDesc, include/skirt_mcrt.h
    _p = ctypes.c_void_p
    _fields_ = [("kind", ctypes.c_int), ("ncells", ctypes.c_int), ("nx", ctypes.c_int), ("ny", ctypes.c_int),
                ("nz", ctypes.c_int), ("xv", _p), ("yv", _p), ("zv", _p), ("nnodes", ctypes.c_int), ("box", _p),
                ("first_child", _p), ("cellnumber", _p), ("nbr_offset", _p), ("nbr_list", _p),
                ("eps", ctypes.c_double), ("search", ctypes.c_int), ("site", _p),
                ("cell_nbr_offset", ctypes.POINTER(ctypes.c_int)), ("cell_nbr_list", ctypes.POINTER(ctypes.c_int)),
                ("cell_bbox", ctypes.POINTER(ctypes.c_double)), ("extent", ctypes.c_double * 6),
                ("nblocks", ctypes.c_int), ("block_offset", ctypes.POINTER(ctypes.c_int)),
                ("block_list", ctypes.POINTER(ctypes.c_int)), ("split_dir", _p)]


def _tessellate(sites, extent, device):
    L = S.lib()
    dp = ctypes.POINTER(ctypes.c_double)
    L.skirt_host_voronoi_build_ex.restype = ctypes.c_void_p
    L.skirt_host_voronoi_build_ex.argtypes = [dp, ctypes.c_int, dp, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    L.skirt_host_voronoi_describe.argtypes = [ctypes.c_void_p, ctypes.POINTER(_GridDesc)]
    L.skirt_host_voronoi_cells.argtypes = [ctypes.c_void_p, dp, dp]
    L.skirt_host_voronoi_free.argtypes = [ctypes.c_void_p]
    sites = np.ascontiguousarray(sites, dtype=np.float64)
    ext = np.ascontiguousarray(extent, dtype=np.float64)
    hc = ctypes.c_int(-1)
    t0 = time.time()
    h = L.skirt_host_voronoi_build_ex(sites.ctypes.data_as(dp), len(sites), ext.ctypes.data_as(dp), device,
                                      ctypes.byref(hc))
    dt = time.time() - t0
    assert h, L.skirt_sim_error().decode()
    try:
        g = _GridDesc()
        assert L.skirt_host_voronoi_describe(h, ctypes.byref(g)) == 0
        n, nb = g.ncells, g.nblocks
        off = np.ctypeslib.as_array(g.cell_nbr_offset, (n + 1,)).copy()
        boff = np.ctypeslib.as_array(g.block_offset, (nb ** 3 + 1,)).copy()
        out = {"nbr_offset": off, "nbr_list": np.ctypeslib.as_array(g.cell_nbr_list, (int(off[-1]),)).copy(),
               "bbox": np.ctypeslib.as_array(g.cell_bbox, (6 * n,)).copy(), "block_offset": boff,
               "block_list": np.ctypeslib.as_array(g.block_list, (int(boff[-1]),)).copy(),
               "volume": np.empty(n), "centroid": np.empty(3 * n)}
        assert L.skirt_host_voronoi_cells(h, out["volume"].ctypes.data_as(dp), out["centroid"].ctypes.data_as(dp)) == 0
    finally:
        L.skirt_host_voronoi_free(h)
    return out, hc.value, dt


def _plummer(n, c, h, seed):
    rng = np.random.default_rng(seed)
    out = []
    while sum(len(o) for o in out) < n:
        t = np.cbrt(rng.random(n))
        r = c * t / np.sqrt((1 - t) * (1 + t))
        ct = 2 * rng.random(n) - 1
        ph = 2 * np.pi * rng.random(n)
        st = np.sqrt(1 - ct * ct)
        p = np.stack([r * st * np.cos(ph), r * st * np.sin(ph), r * ct], axis=1)
        out.append(p[np.all(np.abs(p) <= h, axis=1)])
    return np.concatenate(out)[:n]


@pytest.mark.parametrize("kind,n", [("plummer", 100000), ("uniform", 20000), ("plummer", 37)])
def test_device_voronoi_cells_equal_host(kind, n):
    """skirt_mcrt_voronoi_cells against the host construction on the same sites: neighbour lists, bounding
    boxes, block lists, volumes and centroids bit for bit (the cells that outgrow the device's capacities are
    built on the host; their number is reported)."""
    h = 1.0
    if kind == "plummer":
        sites = _plummer(n, 0.1, h, 7 + n)
    else:
        sites = np.random.default_rng(3).uniform(-h, h, size=(n, 3))
    extent = [-h, -h, -h, h, h, h]
    host, hc0, th = _tessellate(sites, extent, -1)
    dev, hc1, td = _tessellate(sites, extent, 0)
    print("%s %d sites: host %.3f s, device %.3f s (%d cells on the host)" % (kind, n, th, td, hc1))
    assert hc0 == n and 0 <= hc1 <= n // 200
    for k in host:
        assert np.array_equal(host[k], dev[k]), k
