"""ExpDiskGeometry stars and dust on the GPU against the CPU oracle on the same Philox streams (the
geometry's restatement is checked on its own in tests/test_geometries.py; parity unpinned against the
reference itself, which has no fixture for it)."""
import numpy as np
import pytest

import oracle_lib as O
import skirt_amd as S
import tree_models as T
from test_gpu_parity import close_fraction

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["disk_cart", "disk_oct"])
def test_exp_disk_engine_matches_oracle_same_streams(tmp_path, name):
    path = T.write_geometry(name, str(tmp_path))
    packages = 3000
    sim = S.Simulation(path, packages=packages)
    sim.attach(0)
    sim.run_stellar()
    sim.fetch()
    st = sim.stats()
    orc = O.run(path, rng=O.RNG_PHILOX, threads=16, packages=packages)
    assert st["packets"] == orc.packets
    labs = sim.labs()
    np.testing.assert_allclose(labs.sum(), orc.labs.sum(), rtol=1e-9)
    np.testing.assert_allclose(labs.sum(axis=0), orc.labs.sum(axis=0), rtol=1e-9)
    assert close_fraction(labs, orc.labs, 1e-9) > 0.999
    frames, seds = sim.instrument(0)
    np.testing.assert_allclose(seds, orc.seds[0], rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(frames.sum(axis=2), orc.frames[0].sum(axis=2), rtol=1e-9, atol=1e-300)
    assert close_fraction(frames, orc.frames[0], 1e-9) > 0.999
