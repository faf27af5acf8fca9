"""The setup's density sampling on the device (skirt_sim_load_ex / Simulation(setup_device=0), through
skirt_mcrt_sample_density) against the host setup, which is bit-identical to the reference
(tests/test_oracle_golden.py): the same random words, the same tree, and cell densities equal to an ulp
of the device's exp/pow/log10 (relative tolerance 1e-13). Reference: DustSystem::setupSelfAfter
(DustSystem.cpp:152-178), TreeNodeSampleDensityCalculator (TreeDustGrid.cpp:174-222)."""
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
