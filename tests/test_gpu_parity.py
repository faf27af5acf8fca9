"""GPU engine (through the C ABI / host driver) against the CPU oracle and the reference fixtures.

1. Same random streams: the engine and the oracle's Philox mode shoot the same packets with the same
   per-packet Philox streams, so every tally must agree to floating-point rounding. Device libm
   (ocml) and glibc differ in the last ulp of exp/log/pow/trig, which can very rarely flip a discrete
   decision (a cell boundary, a rejection test) and change one packet's history; the tolerances allow
   for that: totals to 1e-9 relative, 99.9 % of the per-cell / per-pixel values to 1e-9 relative.
2. Against the reference itself (`skirt -t 1` outputs in tests/golden/ref): different random streams,
   so per-wavelength absorbed luminosities and fluxes are compared with a z-test whose variance comes
   from several engine runs with independent seeds (sqrt(N) Monte Carlo tolerance).
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import skirt_files as F
import skirt_amd as S
from skirt_amd.sharding import shard_slice

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def ski(name):
    return os.path.join(GOLD, "ski", name + ".ski")


def run_gpu(name, packages=0.0, seed=0, first=0, count=0, dust=False):
    sim = S.Simulation(ski(name), packages=packages, seed=seed)
    sim.attach(0)
    sim.run_stellar(first, count)
    if dust:
        sim.run_dust()
    sim.fetch()
    return sim


def close_fraction(a, b, rtol, floor=1e-15):
    """Fraction of elements equal to rtol; values below floor x the table's maximum are ignored (in
    optically thick models the deepest cells receive ~1e-220 of the packet luminosity, where the
    engine's running exp(-tau) and the oracle's exp(-tau) per segment underflow at different depths)."""
    a, b = np.asarray(a).ravel(), np.asarray(b).ravel()
    scale = np.maximum(np.abs(a), np.abs(b))
    ok = np.abs(a - b) <= rtol * scale + floor * scale.max() + 1e-300
    return ok.mean()


@pytest.mark.parametrize("name,packages", [("c1_oligo16", 20000), ("oligo_2comp", 5000), ("pan_cart16", 3000),
                                           ("pan_oct", 3000), ("vor_oligo", 5000), ("vor_pan", 1000)])
def test_engine_matches_oracle_same_streams(name, packages):
    sim = run_gpu(name, packages=packages)
    orc = O.run(ski(name), rng=O.RNG_PHILOX, threads=16, packages=packages)
    st = sim.stats()
    assert st["packets"] == orc.packets
    if orc.labs is not None:
        labs = sim.labs()
        np.testing.assert_allclose(labs.sum(), orc.labs.sum(), rtol=1e-9)
        np.testing.assert_allclose(labs.sum(axis=0), orc.labs.sum(axis=0), rtol=1e-9)
        assert close_fraction(labs, orc.labs, 1e-9) > 0.999
    for i in range(sim.info.ninstruments):
        frames, seds = sim.instrument(i)
        if seds is not None:
            np.testing.assert_allclose(seds, orc.seds[i], rtol=1e-9, atol=1e-300)
        if frames is not None:
            np.testing.assert_allclose(frames.sum(axis=2), orc.frames[i].sum(axis=2), rtol=1e-9, atol=1e-300)
            assert close_fraction(frames, orc.frames[i], 1e-9) > 0.999


@pytest.mark.parametrize("path,packages", [(os.path.join("tests", "golden", "ski", "pan_oct.ski"), 3000),
                                           (os.path.join("benchmarks", "c3_oct128.ski"), 40)])
def test_leaf_map_walk_equals_node_walk(path, packages, monkeypatch):
    """The octree leaf-map walk takes exactly the reference's steps: the same segment, absorption and
    detection counts as the node-array walk (TreeNode neighbour search), and the same tallies up to the
    order of the f64 atomic additions."""
    full = os.path.join(os.path.dirname(GOLD), "..", path)
    runs = []
    for leafmap in ("1", "0"):
        monkeypatch.setenv("SKIRT_AMD_LEAFMAP", leafmap)
        sim = S.Simulation(full, packages=packages)
        sim.attach(0)
        sim.run_stellar()
        sim.fetch()
        runs.append(sim)
    a, b = runs
    sa, sb = a.stats(), b.stats()
    for k in ("packets", "segments_fill", "segments_walk", "segments_peel", "detects", "absorb_adds"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    np.testing.assert_allclose(a.labs(), b.labs(), rtol=1e-10, atol=1e-300)
    fa, da = a.instrument(0)
    fb, db = b.instrument(0)
    np.testing.assert_allclose(da, db, rtol=1e-10, atol=1e-300)
    np.testing.assert_allclose(fa, fb, rtol=1e-10, atol=1e-300)


@pytest.mark.parametrize("name,packages", [("pan_cart16", 2000), ("pan_oct", 2000), ("pan_cart16_sa", 1000),
                                           ("vor_pan", 1000)])
def test_dust_phases_match_oracle_same_streams(name, packages):
    """Stellar emission, the self-absorption cycles (if the model has them) and the dust emission phase
    (PanMonteCarloSimulation::runSelf) on the GPU against the oracle on the same Philox streams. The
    grey-body spectra and cell sources between phases are host code shared by both, fed each time by
    the engine's own tallies."""
    sim = S.Simulation(ski(name), packages=packages)
    sim.attach(0)
    sim.run_stellar()
    sim.run_dust()
    sim.fetch()
    orc = O.run(ski(name), rng=O.RNG_PHILOX, threads=16, packages=packages, phases=O.PHASES_ALL)
    np.testing.assert_allclose(sim.labs().sum(axis=0), orc.labs.sum(axis=0), rtol=1e-9)
    assert close_fraction(sim.labs(), orc.labs, 1e-9) > 0.999
    if orc.labs_dust is not None:
        totals = sim.selfabs_totals()
        assert len(totals) == len(orc.labs_dust_totals)
        np.testing.assert_allclose(totals, orc.labs_dust_totals, rtol=1e-8)
        np.testing.assert_allclose(sim.labs_dust().sum(axis=0), orc.labs_dust.sum(axis=0), rtol=1e-8)
        assert close_fraction(sim.labs_dust(), orc.labs_dust, 1e-8) > 0.99
    frames, seds = sim.instrument(0)
    assert seds[3:5].sum() > 0  # dust direct and dust scattered slots received the dust emission
    np.testing.assert_allclose(seds, orc.seds[0], rtol=1e-8, atol=1e-300)
    np.testing.assert_allclose(frames.sum(axis=2), orc.frames[0].sum(axis=2), rtol=1e-8, atol=1e-300)
    assert close_fraction(frames, orc.frames[0], 1e-8) > 0.99


@pytest.mark.parametrize("name", ["pan_oct", "pan_cart16_sa"])
def test_device_cell_sources_equal_host_cell_sources(name, monkeypatch):
    """The grey-body spectra and cell distributions computed on the device between phases give the
    same dust phases as the host restatement shared with the oracle (to rounding)."""
    runs = []
    for host in ("0", "1"):
        monkeypatch.setenv("SKIRT_AMD_HOST_SOURCES", host)
        runs.append(run_gpu(name, packages=1000, dust=True))
    dev, host = runs
    np.testing.assert_allclose(dev.selfabs_totals(), host.selfabs_totals(), rtol=1e-9)
    fd, sd = dev.instrument(0)
    fh, sh = host.instrument(0)
    np.testing.assert_allclose(sd, sh, rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(fd.sum(axis=2), fh.sum(axis=2), rtol=1e-9, atol=1e-300)


def test_sharded_packet_ranges_sum_to_the_whole():
    """Two disjoint packet ranges (as two GPUs would run) add up to the full run exactly."""
    name = "pan_cart16"
    full = run_gpu(name, packages=2000)
    total = full.info.total_packets
    a = run_gpu(name, packages=2000, first=0, count=total // 3)
    b = run_gpu(name, packages=2000, first=total // 3, count=total - total // 3)
    np.testing.assert_allclose(a.labs() + b.labs(), full.labs(), rtol=1e-12, atol=1e-300)
    fa, sa = a.instrument(0)
    fb, sb = b.instrument(0)
    ff, sf = full.instrument(0)
    np.testing.assert_allclose(sa + sb, sf, rtol=1e-12)
    np.testing.assert_allclose(fa + fb, ff, rtol=1e-12, atol=1e-300)


def test_wavelength_shards_sum_to_the_whole():
    """Three ranks' slices of every wavelength (skirt_mcrt_run_phase_shard, the reference's
    IdenticalAssigner) add up to the full run exactly, and each rank shoots every wavelength."""
    name = "pan_cart16"
    full = run_gpu(name, packages=2000)
    parts = []
    for r in range(3):
        sim = S.Simulation(ski(name), packages=2000)
        sim.attach(0)
        calls = []
        sim.set_reducer(lambda tally, ptr, n, stream: calls.append(tally))  # single process: no sum
        sim.run_stellar_shard(r, 3)
        sim.fetch()
        assert calls == [S.TALLY_LABS, S.TALLY_INSTRUMENTS]
        lo, n = shard_slice(2000, r, 3)
        assert sim.stats()["packets"] == n * np.count_nonzero(full.labs().sum(axis=0) > 0)
        assert np.all(sim.labs().sum(axis=0)[full.labs().sum(axis=0) > 0] > 0)
        parts.append(sim)
    np.testing.assert_allclose(sum(p.labs() for p in parts), full.labs(), rtol=1e-12, atol=1e-300)
    ff, sf = full.instrument(0)
    np.testing.assert_allclose(sum(p.instrument(0)[1] for p in parts), sf, rtol=1e-12)
    np.testing.assert_allclose(sum(p.instrument(0)[0] for p in parts), ff, rtol=1e-12, atol=1e-300)
    with pytest.raises(S.SkirtError, match="summed"):
        parts[0].run_stellar_shard(0, 3)  # the instruments were summed: a further phase is refused


def _isrf_sums(path):
    """Per-wavelength sum over cells of the mean intensity J in a ds_isrf file. J is Labs divided by a
    per-(cell, wavelength) constant of the model (DustSystem::meanintensityv), so these sums are linear
    Monte Carlo estimators with the same expectation for the engine and the reference."""
    return F.read_text_table(path)[:, 4:].sum(axis=0)


@pytest.mark.parametrize("name", ["pan_cart16", "pan_oct", "pan_cart16_sa", "vor_pan"])
def test_engine_matches_reference_statistically(tmp_path, name):
    """All phases (stellar, self-absorption, dust emission) against `skirt -t 1`: per-wavelength ISRF sums
    and every SED column -- total, direct and scattered stellar, dust emission, dust scattered,
    transparent -- as z-scores against the spread of 8 independently seeded engine runs."""
    seeds = [101, 202, 303, 404, 505, 606, 707, 808]
    Jsum, seds = [], []
    for k, sd in enumerate(seeds):
        r = run_gpu(name, seed=sd, dust=True)
        prefix = str(tmp_path / ("%s_%d" % (name, k)))
        r.write(prefix)
        Jsum.append(_isrf_sums(prefix + "_ds_isrf.dat"))
        seds.append(F.read_text_table(prefix + "_i30_sed.dat"))
    Jsum, seds = np.array(Jsum), np.array(seds)
    ref_J = _isrf_sums(os.path.join(GOLD, "ref", name + "_s4357_ds_isrf.dat"))
    ref_sed = F.read_text_table(os.path.join(GOLD, "ref", name + "_s4357_i30_sed.dat"))
    infl = np.sqrt(1 + 1.0 / len(seeds))
    m, s = Jsum.mean(axis=0), Jsum.std(axis=0, ddof=1)
    good = s > 0
    z = (ref_J[good] - m[good]) / (s[good] * infl)
    assert np.all(np.abs(z) < 5), z
    for col in (1, 2, 3, 4, 5, 6):  # total, direct, scattered, dust, dust scattered, transparent
        m, s = seds[:, :, col].mean(axis=0), seds[:, :, col].std(axis=0, ddof=1)
        good = s > 0
        zz = (ref_sed[good, col] - m[good]) / (s[good] * infl)
        assert np.all(np.abs(zz) < 5), (col, zz)


def test_transparent_flux_is_deterministic():
    """F_trav = L/(4 pi d^2) for any seed (invariant 4): 2.41996378e-12 W/m2."""
    sim = run_gpu("c1_oligo16", packages=30000, seed=5)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        sim.write(os.path.join(d, "t"))
        sed = F.read_text_tokens(os.path.join(d, "t_i30_sed.dat"))
    assert sed[0][6] == "2.41996378e-12"
