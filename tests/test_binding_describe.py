"""The maintainer binding's data extraction, executed (the binding itself is
integration/GpuPhotonEngine.cpp). integration/build_describe.sh links the binding with the
reference's own objects (oracle/ref.mk, built from /root/reference); integration/describe_main.cpp sets a .ski
up through the reference's XmlHierarchyCreator and Simulation::setup (on one thread, as `skirt -t 1`) and
writes the descriptors the binding builds from the live simulation items -- the tree's `_tree`,
`_cellnumberv` and neighbour lists, the Voronoi mesh's sites, DustSystem::density, DustMix's tables and
`_asymmparv`, the stellar components and geometries, the instruments (DustGrid.hpp:70-106,
DustSystem.hpp:352-397, Instrument.hpp:69-87) -- instead of uploading them. skirt_sim_describe writes what the
.ski driver uploads for the same file. The two dumps must agree bit for bit, field by field: the binding
would hand the engine exactly what the parity tests run. Needs /root/reference (the build container), no GPU."""
import os
import subprocess

import numpy as np
import pytest

import descriptors as D
import skirt_amd as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
GOLD = os.path.join(REPO, "tests", "golden", "ski")
HARNESS = os.path.join(REPO, "integration", "_build", "describe")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "SKIRTcore")),
                                reason="needs the reference sources (build container)")

MODELS = ["pan_cart16", "pan_oct", "vor_pan", "c1_oligo16", "oligo_2comp", "bin_pan", "oct_bary", "oct_pan_bk",
          "cart_pow", "disk_oct", "sersic_cart", "point_cart", "draineli_cart", "bbody_cart", "edgeon_cart",
          "bench:c3_oct128", "bench:c4_vor1e5"]


@pytest.fixture(scope="module")
def harness():
    subprocess.run(["bash", os.path.join(REPO, "integration", "build_describe.sh")], check=True,
                   capture_output=True, timeout=1800)
    return HARNESS


def _ski(name, tmp_path):
    if name.startswith("bench:"):
        return os.path.join(REPO, "benchmarks", name[6:] + ".ski")
    path = os.path.join(GOLD, name + ".ski")
    if os.path.exists(path):
        return path
    import tree_models
    return tree_models.write_any(name, str(tmp_path))


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", MODELS)
def test_binding_describes_the_model_as_the_ski_driver_does(harness, tmp_path, name):
    ski = _ski(name, tmp_path)
    ours, binding = str(tmp_path / "driver.bin"), str(tmp_path / "binding.bin")
    S.Simulation(ski).describe(ours)
    r = subprocess.run([harness, ski, binding, str(tmp_path)], capture_output=True, text=True, timeout=850)
    assert r.returncode == 0, r.stderr[-2000:]
    a, b = D.read(ours), D.read(binding)
    diffs = D.differences(a, b)
    if a["grid.kind"][0] == S.GRID_VORONOI:
        # DustSystem samples a Voronoi cell's density at random points of the cell's bounding box
        # (VoronoiMesh::randomPosition), which the reference takes from Voro++ and the host driver from its
        # own clipping of the same cell (the binding re-tessellates the sites with it too, so the grid fields
        # agree bit for bit): the sample points, and so the sampled densities, differ in their last digits
        assert [k for k, _ in diffs] in ([], ["media.rho"]), diffs
        np.testing.assert_allclose(b["media.rho"], a["media.rho"], rtol=1e-12, atol=0)
    else:
        assert diffs == []
    # the dumps hold the model: cells, densities, sources, instruments
    assert a["grid.ncells"][0] > 0 and a["media.rho"].sum() > 0
    assert a["sources.lumtot"].sum() > 0 and a["instruments.n"][0] >= 1
