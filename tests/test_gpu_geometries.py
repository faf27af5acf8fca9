"""ExpDiskGeometry and SersicGeometry stars and dust on the GPU against the CPU oracle on the same Philox
streams (the geometries' restatements are checked on their own in tests/test_geometries.py; parity
pinned against the reference by the disk_oct, disk_cart, bulge_oct, sersic_cart and point_oct fixtures)."""
import os

import numpy as np
import pytest

import oracle_lib as O
import skirt_amd as S
import tree_models as T
from parity import DUST_OUTLIERS, STELLAR_OUTLIERS, assert_parity

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["disk_cart", "disk_oct", "bulge_oct", "sersic_cart", "point_oct", "point_cart"])
def test_geometry_engine_matches_oracle_same_streams(tmp_path, name):
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
    assert_parity(labs, orc.labs, 1e-9, STELLAR_OUTLIERS, "labs")
    frames, seds = sim.instrument(0)
    np.testing.assert_allclose(seds, orc.seds[0], rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(frames.sum(axis=2), orc.frames[0].sum(axis=2), rtol=1e-9, atol=1e-300)
    assert_parity(frames, orc.frames[0], 1e-9, STELLAR_OUTLIERS, "frames")


def test_dust_free_blackbody_engine_matches_oracle(tmp_path):
    """A dust-free model (every packet ends at its emission peel-off, detected by the event kernel)
    with a BlackBodySED, a FullInstrument and an SEDInstrument: the engine's tallies equal the oracle's
    on the same streams."""
    from test_seds import SKI
    full = ('<FullInstrument instrumentName="f" distance="10 Mpc" inclination="60 deg" azimuth="0 deg" '
            'positionAngle="0 deg" fieldOfViewX="1000 pc" pixelsX="24" centerX="0 pc" fieldOfViewY="1000 pc" '
            'pixelsY="20" centerY="0 pc" scatteringLevels="2"/>')
    text = SKI % {"N": 12, "SED": '<BlackBodySED temperature="8000 K"/>'}
    text = text.replace("<SEDInstrument", full + "\n            <SEDInstrument")
    path = str(tmp_path / "bb_free.ski")
    with open(path, "w") as f:
        f.write(text)
    packages = 20000
    sim = S.Simulation(path, packages=packages)
    sim.attach(0)
    sim.run_stellar()
    sim.fetch()
    orc = O.run(path, rng=O.RNG_PHILOX, threads=16, packages=packages)
    assert sim.stats()["packets"] == orc.packets
    for i in range(2):
        frames, seds = sim.instrument(i)
        np.testing.assert_allclose(seds, orc.seds[i], rtol=1e-12, atol=1e-300)
        if orc.frames[i] is not None and orc.frames[i].size:
            np.testing.assert_allclose(frames.sum(axis=2), orc.frames[i].sum(axis=2), rtol=1e-9, atol=1e-300)
            assert_parity(frames, orc.frames[i], 1e-9, STELLAR_OUTLIERS, "frames")


@pytest.mark.parametrize("name", ["zubko_cart", "draineli_cart"])
def test_dust_mix_engine_matches_oracle_same_streams(tmp_path, name):
    path = T.write_mix(name, str(tmp_path))
    packages = 3000
    sim = S.Simulation(path, packages=packages)
    sim.attach(0)
    sim.run_stellar()
    sim.fetch()
    orc = O.run(path, rng=O.RNG_PHILOX, threads=16, packages=packages)
    assert sim.stats()["packets"] == orc.packets
    labs = sim.labs()
    np.testing.assert_allclose(labs.sum(axis=0), orc.labs.sum(axis=0), rtol=1e-9)
    assert_parity(labs, orc.labs, 1e-9, STELLAR_OUTLIERS, "labs")
    frames, seds = sim.instrument(0)
    np.testing.assert_allclose(seds, orc.seds[0], rtol=1e-9, atol=1e-300)


def test_cli_runs_every_phase(tmp_path):
    """skirt-mi355x (SkirtMain's counterpart) runs the stellar phase, the self-absorption cycles and the dust
    emission phase of a Pan model and writes SKIRT's outputs with the dust columns filled."""
    import subprocess

    import skirt_files as F

    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "skirt_amd", "bin", "skirt-mi355x")
    ski = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ski", "pan_cart16_sa.ski")
    prefix = str(tmp_path / "sa")
    r = subprocess.run([exe, "-p", "500", "-o", prefix, ski], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("Self-absorption cycle") == 6, r.stdout
    sed = F.read_text_table(prefix + "_i30_sed.dat")
    assert sed[:, 4].sum() > 0 and sed[:, 5].sum() > 0  # dust emission: direct and scattered
    assert os.path.exists(prefix + "_ds_isrf.dat")
