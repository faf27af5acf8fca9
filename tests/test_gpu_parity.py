"""GPU engine (through the C ABI / host driver) against the CPU oracle and the reference fixtures.

1. Same random streams: the engine and the oracle's Philox mode shoot the same packets with the same
   per-packet Philox streams, so every tally must agree to floating-point rounding. Device libm
   (ocml) and glibc differ in the last ulp of exp/log/pow/trig, which can very rarely flip a discrete
   decision (a cell boundary, a rejection test) and change one packet's history; the tolerances allow
   for that: totals to 1e-9 relative, per-cell / per-pixel values to 1e-9 relative with an explicit
   outlier budget (tests/parity.py: count and mass of the outliers).
2. Against the reference itself (`skirt -t 1` outputs in tests/golden/ref): different random streams,
   so per-wavelength absorbed luminosities and fluxes are compared with a z-test whose variance comes
   from several engine runs with independent seeds (sqrt(N) Monte Carlo tolerance).
"""
import os
import re

import numpy as np
import pytest

import oracle_lib as O
from parity import DUST_OUTLIERS, STELLAR_OUTLIERS, assert_parity
import skirt_files as F
import skirt_amd as S
from skirt_amd.sharding import shard_slice

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def ski(name):
    path = os.path.join(GOLD, "ski", name + ".ski")
    if not os.path.exists(path):  # a variant of tests/tree_models.py (grid, geometry, mix, outputs)
        import tempfile
        import tree_models
        path = tree_models.write_any(name, tempfile.mkdtemp(prefix="skirt_variant_"))
    return path


def run_gpu(name, packages=0.0, seed=0, first=0, count=0, dust=False):
    sim = S.Simulation(ski(name), packages=packages, seed=seed)
    sim.attach(0)
    sim.run_stellar(first, count)
    if dust:
        sim.run_dust()
    sim.fetch()
    return sim


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
        assert_parity(labs, orc.labs, 1e-9, STELLAR_OUTLIERS, "labs")
    for i in range(sim.info.ninstruments):
        frames, seds = sim.instrument(i)
        if seds is not None:
            np.testing.assert_allclose(seds, orc.seds[i], rtol=1e-9, atol=1e-300)
        if frames is not None:
            np.testing.assert_allclose(frames.sum(axis=2), orc.frames[i].sum(axis=2), rtol=1e-9, atol=1e-300)
            assert_parity(frames, orc.frames[i], 1e-9, STELLAR_OUTLIERS, "frames")


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


@pytest.mark.parametrize("name,packages,dust", [("pan_cart16", 2000, False), ("pan_oct", 2000, False),
                                                ("vor_pan", 1000, False), ("pan_oct_sa", 500, True),
                                                ("vor_pan_cs", 150, False)])
def test_walk_ray_queue_order_does_not_change_results(name, packages, dust, monkeypatch):
    """WALK rays queued from the top of the ray queue and pulled last (SKIRT_AMD_WALK_BACK=1, the Voronoi
    default) or in event order (0, the tree and Cartesian default): the same packets take the same paths,
    so the counts are equal and the tallies agree up to the order of the f64 atomic additions."""
    runs = []
    for back in ("1", "0"):
        monkeypatch.setenv("SKIRT_AMD_WALK_BACK", back)
        runs.append(run_gpu(name, packages=packages, dust=dust))
    _assert_same_packets(*runs)


@pytest.mark.parametrize("name,packages,dust", [("pan_oct", 2000, False), ("pan_oct_sa", 500, True),
                                                ("pan_oct_cs", 200, True), ("pan_cart16_sa", 500, True),
                                                ("vor_pan", 1000, False), ("vor_pan_cs", 150, False),
                                                ("oligo_2comp", 3000, False)])
def test_global_atomic_kernels_equal_buffer_atomic_kernels(name, packages, dust, monkeypatch):
    """The trace kernels of a Labs table of 4 GiB or more (global atomics, their own instantiations since round
    6: Tracer GLOBAL) against the buffer-atomic kernels, forced by SKIRT_AMD_LABS_GLOBAL=1 on small tables, for
    each family: octree leaf map, Cartesian, Voronoi, continuous scattering, the dust phases, several dust
    components. The same packets take the same paths; the tallies agree up to the order of the additions."""
    runs = []
    for glob in ("1", "0"):
        monkeypatch.setenv("SKIRT_AMD_LABS_GLOBAL", glob)
        runs.append(run_gpu(name, packages=packages, dust=dust))
    _assert_same_packets(*runs)


@pytest.mark.parametrize("name,packages,dust", [("pan_cart16", 2000, False), ("pan_oct", 2000, True),
                                                ("vor_pan", 1000, False)])
def test_two_pipeline_halves_do_not_change_results(name, packages, dust, monkeypatch):
    """The slot pool as two independent pipelines (SKIRT_AMD_HALVES=2: one half's event and detect kernels
    beside the other half's trace kernel, on CU-masked streams, SKIRT_AMD_TRACE_CUS / SKIRT_AMD_EVENT_CUS
    CUs each) against one: packets are claimed from one counter either way, so the same packets take the
    same paths and the tallies agree up to the order of the atomic additions."""
    runs = []
    for halves, cus in (("2", "192"), ("1", "0")):
        monkeypatch.setenv("SKIRT_AMD_HALVES", halves)
        monkeypatch.setenv("SKIRT_AMD_TRACE_CUS", cus)
        monkeypatch.setenv("SKIRT_AMD_EVENT_CUS", "64" if halves == "2" else "0")
        runs.append(run_gpu(name, packages=packages, dust=dust))
    _assert_same_packets(*runs)


@pytest.mark.parametrize("name,packages", [("pan_oct_sa", 1000), ("pan_cart16", 2000), ("bin_pan", 1000)])
def test_no_store_trace_kernel_does_not_change_results(name, packages, monkeypatch):
    """The dust emission phase stores no absorption; with one component it runs traceKernelNoStore (no Labs
    buffers, 4 waves per SIMD). SKIRT_AMD_NO_NOSTORE=1 runs it on the storing kernel instead: the same
    packets, the same paths, tallies equal up to the order of the atomic additions."""
    runs = []
    for off in ("0", "1"):
        if off == "1":
            monkeypatch.setenv("SKIRT_AMD_NO_NOSTORE", "1")
        else:
            monkeypatch.delenv("SKIRT_AMD_NO_NOSTORE", raising=False)
        runs.append(run_gpu(name, packages=packages, dust=True))
    # the last phase (dust emission) ran at the no-store kernel's occupancy: more trace blocks per CU
    assert runs[0].stats()["trace_blocks_per_cu"] > runs[1].stats()["trace_blocks_per_cu"]
    _assert_same_packets(*runs)


@pytest.mark.parametrize("name,packages,dust", [("pan_oct_sa", 1000, True), ("c1_oligo16", 20000, False)])
def test_labs_replicas_do_not_change_results(name, packages, dust, monkeypatch):
    """The absorbing phases add into replicas of the Labs table, folded into it at the phase end (by default
    as many as fit 320 MiB, at most 8); SKIRT_AMD_LABS_COPIES=1 adds into the table itself and =3 into three
    replicas: the same packets, tallies equal up to the order of the additions."""
    runs = []
    for k in (None, "1", "3"):
        if k is None:
            monkeypatch.delenv("SKIRT_AMD_LABS_COPIES", raising=False)
        else:
            monkeypatch.setenv("SKIRT_AMD_LABS_COPIES", k)
        runs.append(run_gpu(name, packages=packages, dust=dust))
    _assert_same_packets(runs[1], runs[0])
    _assert_same_packets(runs[1], runs[2])


def _assert_same_packets(a, b):
    sa, sb = a.stats(), b.stats()
    for k in ("packets", "segments_fill", "segments_walk", "segments_peel", "detects", "absorb_adds"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    for la, lb in ((a.labs(), b.labs()), (a.labs_dust(), b.labs_dust())):
        assert (la is None) == (lb is None)
        if la is not None:
            np.testing.assert_allclose(la, lb, rtol=1e-10, atol=1e-300)
    for i in range(a.info.ninstruments):
        fa, da = a.instrument(i)
        fb, db = b.instrument(i)
        if da is not None:
            np.testing.assert_allclose(da, db, rtol=1e-10, atol=1e-300)
        if fa is not None:
            np.testing.assert_allclose(fa, fb, rtol=1e-10, atol=1e-300)


@pytest.mark.parametrize("name,packages", [("pan_cart16", 2000), ("pan_oct", 2000), ("pan_cart16_sa", 1000),
                                           ("pan_oct_sa", 1000), ("pan_oct_sac", 1000), ("vor_pan", 1000),
                                           ("pan_cart16_cs", 300), ("pan_oct_cs", 300), ("vor_pan_cs", 200)])
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
    # (the optically thick pan_oct_sa models included: exp(-tau) per segment as the reference, tests/parity.py)
    assert_parity(sim.labs(), orc.labs, 1e-9, STELLAR_OUTLIERS, "labs")
    if orc.labs_dust is not None:
        totals = sim.selfabs_totals()
        assert len(totals) == len(orc.labs_dust_totals)
        np.testing.assert_allclose(totals, orc.labs_dust_totals, rtol=1e-8)
        np.testing.assert_allclose(sim.labs_dust().sum(axis=0), orc.labs_dust.sum(axis=0), rtol=1e-8)
        assert_parity(sim.labs_dust(), orc.labs_dust, 1e-8, DUST_OUTLIERS, "labs_dust")
    frames, seds = sim.instrument(0)
    assert seds[3:5].sum() > 0  # dust direct and dust scattered slots received the dust emission
    np.testing.assert_allclose(seds, orc.seds[0], rtol=1e-8, atol=1e-300)
    np.testing.assert_allclose(frames.sum(axis=2), orc.frames[0].sum(axis=2), rtol=1e-8, atol=1e-300)
    assert_parity(frames, orc.frames[0], 1e-8, DUST_OUTLIERS, "frames")


@pytest.mark.parametrize("name", ["pan_oct", "pan_cart16_sa", "pan_oct_sa"])
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


@pytest.mark.parametrize("name,mix", [("c1_oligo16", "OligoDustSystem"), ("pan_cart16", "PanDustSystem")])
def test_dust_free_models_match_oracle_same_streams(tmp_path, name, mix):
    """A simulation without a dust system (MonteCarloSimulation.cpp:265-301 with _ds null): every packet is
    launched, detected unattenuated by every instrument and ends in the event kernel (no trace kernel, no
    Labs). Engine = oracle on the same Philox streams."""
    text = open(ski(name)).read()
    text, n = re.subn(r'\s*<dustSystem type="%s">.*?</dustSystem>' % mix, "", text, flags=re.S)
    assert n == 1
    path = str(tmp_path / (name + "_nodust.ski"))
    with open(path, "w") as f:
        f.write(text)
    packages = 2000
    sim = S.Simulation(path, packages=packages)
    assert sim.info.has_dust == 0
    sim.attach(0)
    sim.run_stellar()
    sim.run_dust()
    sim.fetch()
    orc = O.run(path, rng=O.RNG_PHILOX, threads=16, packages=packages, phases=O.PHASES_ALL)
    st = sim.stats()
    assert st["packets"] == orc.packets > 0
    assert st["segments_fill"] == st["segments_walk"] == st["segments_peel"] == 0
    frames, seds = sim.instrument(0)
    np.testing.assert_allclose(seds, orc.seds[0], rtol=1e-12, atol=1e-300)
    if frames is not None:
        np.testing.assert_allclose(frames, orc.frames[0], rtol=1e-12, atol=1e-300)


@pytest.mark.parametrize("name", ["c1_oligo16", "pan_oct", "pan_oct_sac"])
def test_zero_packages_give_zero_tallies(tmp_path, name):
    """A .ski with packages="0": the reference runs no chunk in any phase and writes zeros (the oracle
    restates it); the engine runs every phase empty, the self-absorption cycles and the dust emission
    included, and its tallies are zero, not NaN."""
    text = open(ski(name)).read()
    text, n = re.subn(r'packages="[^"]*"', 'packages="0"', text)
    assert n >= 1
    path = str(tmp_path / (name + "_p0.ski"))
    with open(path, "w") as f:
        f.write(text)
    sim = S.Simulation(path)
    assert sim.info.npp == 0
    sim.attach(0)
    sim.run_stellar()
    sim.run_dust()
    sim.fetch()
    orc = O.run(path, rng=O.RNG_PHILOX, threads=4, phases=O.PHASES_ALL)
    assert sim.stats()["packets"] == orc.packets == 0
    if sim.info.store_absorption:
        assert np.all(sim.labs() == 0)
    for i in range(sim.info.ninstruments):
        frames, seds = sim.instrument(i)
        for got, want in ((seds, orc.seds[i]), (frames, orc.frames[i])):
            if got is not None:
                assert np.all(got == 0) and np.all(np.asarray(want) == 0)


def test_more_ranks_than_packets_per_wavelength():
    """Ragged shards: 7 ranks over 3 packets per wavelength, so four ranks shoot nothing. Every rank runs its
    (possibly empty) slice of every wavelength without error, and the slices add up to the whole."""
    name = "pan_oct"
    full = run_gpu(name, packages=3)
    parts = []
    for rank in range(7):
        sim = S.Simulation(ski(name), packages=3)
        sim.attach(0)
        sim.set_reducer(lambda tally, ptr, n, stream: None)  # one process: the test sums
        sim.run_stellar_shard(rank, 7)
        sim.fetch()
        parts.append(sim)
    counts = [p.stats()["packets"] for p in parts]
    assert sum(counts) == full.stats()["packets"] and counts.count(0) >= 4, counts
    np.testing.assert_allclose(sum(p.labs() for p in parts), full.labs(), rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(sum(p.instrument(0)[1] for p in parts), full.instrument(0)[1], rtol=1e-12,
                               atol=1e-300)


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


def _isrf_cells(path, ncells):
    """Per-cell J_lambda [ncells, nlambda] of a ds_isrf file (cells with no absorption are not listed: 0)."""
    t = F.read_text_table(path)
    J = np.zeros((ncells, t.shape[1] - 4))
    J[t[:, 0].astype(np.int64)] = t[:, 4:]
    return J


# the engine runs behind each reference comparison: the reference value is then a t variate with 15 degrees of
# freedom in z = (ref - mean) / (sd * sqrt(1 + 1/K)); over the ~1,000 compared elements of the statistical
# test, P(|t_15| > 7) = 4.6e-6 each (8 runs and a bound of 5 left ~1.6 chance exceedances per suite run).
# Elements whose runs spread by more than half their mean are a few packets' events (the UV direct flux through
# an optically thick disk, the Wien tail of the dust emission): heavy-tailed, so no z applies to them; the
# same-stream tests against the oracle (which equals the reference bit for bit on these fixtures) cover them.
SEEDS = [101 * (k + 1) for k in range(16)]
Z_BOUND = 7.0


def _engine_seed_runs(tmp_path, name, seeds=SEEDS):
    """All phases of `name` on the grid of the ski's own seed (the reference run's grid) with independent
    photon streams per seed, written in SKIRT format: (per-cell J [K, ncells, nlambda], SED tables
    [K, nlambda, ncols])."""
    J, seds = [], []
    for k, sd in enumerate(seeds):
        r = S.Simulation(ski(name))  # the ski's setup seed: the reference's grid (octrees depend on it)
        r.set_photon_seed(sd)
        r.attach(0)
        r.run_stellar()
        r.run_dust()
        r.fetch()
        prefix = str(tmp_path / ("%s_%d" % (name, k)))
        r.write(prefix)
        J.append(_isrf_cells(prefix + "_ds_isrf.dat", r.info.ncells))
        seds.append(F.read_text_table(prefix + "_i30_sed.dat"))
    return np.array(J), np.array(seds)


def _reference_outputs(name):
    """(ds_isrf path, SED path) of `skirt -t 1` for `name`: the committed reference fixture (written by the
    reference rebuilt from its sources, tests/golden/make_fixtures.sh; regenerated by
    tests/test_reference_rebuild.py)."""
    ref = os.path.join(GOLD, "ref", name + "_s4357")
    assert os.path.exists(ref + "_ds_isrf.dat") and os.path.exists(ref + "_i30_sed.dat"), name
    return ref + "_ds_isrf.dat", ref + "_i30_sed.dat"


# every fixture model with dust emission (an ISRF): the originals, the C5 shape (octree + self-absorption,
# fixed and convergence-driven cycles), continuous scattering, and the grid / geometry / mix variants
STATISTICAL_MODELS = ["pan_cart16", "pan_oct", "pan_cart16_sa", "vor_pan", "pan_oct_sa", "pan_oct_sac",
                      "pan_cart16_cs", "pan_oct_cs", "vor_pan_cs", "bin_pan", "oct_bary", "oct_pan_bk",
                      "disk_oct", "bulge_oct", "sersic_cart", "cart_pow", "zubko_cart", "draineli_cart",
                      "bbody_cart", "quasar_cart", "faceon_cart", "edgeon_cart", "radial_cart"]


@pytest.mark.parametrize("name", STATISTICAL_MODELS)
def test_engine_matches_reference_statistically(tmp_path, name):
    """All phases (stellar, self-absorption, dust emission) against `skirt -t 1`: per-wavelength ISRF sums
    and every SED column -- total, direct and scattered stellar, dust emission, dust scattered,
    transparent -- as z-scores against the spread of 16 independently seeded engine runs."""
    J, seds = _engine_seed_runs(tmp_path, name)
    Jsum = J.sum(axis=1)
    ref_isrf, ref_sed_path = _reference_outputs(name)
    ref_J = _isrf_sums(ref_isrf)
    ref_sed = F.read_text_table(ref_sed_path)
    infl = np.sqrt(1 + 1.0 / len(SEEDS))
    m, s = Jsum.mean(axis=0), Jsum.std(axis=0, ddof=1)
    good = (s > 0) & (s <= 0.5 * m)
    z = (ref_J[good] - m[good]) / (s[good] * infl)
    assert np.all(np.abs(z) < Z_BOUND), z
    _assert_aggregate(z, "ISRF sums")
    for col in (1, 2, 3, 4, 5, 6):  # total, direct, scattered, dust, dust scattered, transparent
        m, s = seds[:, :, col].mean(axis=0), seds[:, :, col].std(axis=0, ddof=1)
        # values below 1e-12 of the column's peak are the Wien tail of the dust emission (e.g. 1.8e-135 W/m2 at
        # 0.77 micron against a 1.3e-15 peak): set by the few hottest cells, heavy-tailed from run to run (the
        # reference's own pan_oct and pan_oct_cs runs differ there by a factor 340), so no z-score applies
        good = (s > 0) & (m > 1e-12 * m.max()) & (s <= 0.5 * m)
        zz = (ref_sed[good, col] - m[good]) / (s[good] * infl)
        assert np.all(np.abs(zz) < Z_BOUND), (col, zz)
        _assert_aggregate(zz, "SED column %d" % col)


def _assert_aggregate(z, what):
    """An aggregate bound over one output's wavelengths (a chi^2 per degree of freedom), beside the per-wavelength
    |z| < Z_BOUND: the reference value is a t-variate with nu = K - 1 degrees of freedom in each z, so mean z^2
    has E = nu / (nu - 2) and, over n independent wavelengths, an sd of sd(z^2) / sqrt(n) (t_15: 1.154 and
    1.84). Bounded at E + 5 sd: a systematic offset of ~1 sd in every wavelength fails it, which no single z
    does. (Wavelengths of the dust columns share their cells' temperatures, hence the 5 rather than 3.)"""
    n = len(z)
    if n < 5:
        return
    nu = len(SEEDS) - 1
    e2 = nu / (nu - 2)
    sd2 = np.sqrt(3 * nu * nu / ((nu - 2) * (nu - 4)) - e2 * e2)
    chi2 = float(np.mean(np.asarray(z) ** 2))
    assert chi2 < e2 + 5 * sd2 / np.sqrt(n), (what, n, chi2)


def _pools(J, max_rel_sd):
    """Groups the cells of one wavelength into pools of consecutive cell numbers (spatial neighbours in
    the reference's numbering) whose summed J has a relative spread over the seeded runs of at most
    max_rel_sd: well-sampled cells stand alone, sparsely hit cells are pooled until their sum is
    Gaussian enough for a z-score. J: [K, ncells]; returns the list of cell-index arrays."""
    pools, cur = [], []
    acc = np.zeros(J.shape[0])
    for c in range(J.shape[1]):
        if not J[:, c].any():
            continue
        cur.append(c)
        acc += J[:, c]
        mu = acc.mean()
        if mu > 0 and acc.std(ddof=1) <= max_rel_sd * mu:
            pools.append(np.array(cur))
            cur, acc = [], np.zeros(J.shape[0])
    if cur and pools:
        pools[-1] = np.concatenate([pools[-1], np.array(cur)])
    elif cur:
        pools.append(np.array(cur))
    return pools


@pytest.mark.parametrize("name", ["pan_cart16", "pan_oct", "vor_pan", "pan_cart16_sa", "pan_oct_sa"])
def test_per_cell_mean_intensity_matches_reference(tmp_path, name):
    """north_star's per-cell criterion: every cell's J_lambda (ds_isrf, i.e. its absorbed luminosity
    divided by the cell constant of DustSystem::meanintensityv, DustSystem.cpp:935-957) within the Monte
    Carlo spread of the reference's `skirt -t 1` value. Cells are pooled until their summed J is sampled
    well (relative spread <= 25 % over 16 seeded engine runs); the reference value of a pool is then a
    t-variate with 15 degrees of freedom in z = (ref - mean) / (sd * sqrt(1 + 1/K)): E[z^2] = 15/13.
    The test bounds the mean z^2 over all pools (a chi^2 per degree of freedom) and the tail count."""
    seeds = [1000 + 37 * k for k in range(16)]
    J, _ = _engine_seed_runs(tmp_path, name, seeds)
    ref = _isrf_cells(os.path.join(GOLD, "ref", name + "_s4357_ds_isrf.dat"), J.shape[1])
    K = len(seeds)
    infl = np.sqrt(1 + 1.0 / K)
    z = []
    for ell in range(J.shape[2]):
        for p in _pools(J[:, :, ell], 0.25):
            tot = J[:, p, ell].sum(axis=1)
            m, s = tot.mean(), tot.std(ddof=1)
            if s > 0:
                z.append((ref[p, ell].sum() - m) / (s * infl))
    z = np.array(z)
    nu = K - 1
    chi2 = float(np.mean(z ** 2))
    tail = int(np.count_nonzero(np.abs(z) > 4))
    print("per-cell J %s: %d pools, mean z^2 %.3f (t_%d: %.3f), |z|>4: %d" % (name, len(z), chi2, nu, nu / (nu - 2),
                                                                             tail))
    assert len(z) > 100
    # t_15: E[z^2] = 1.154, sd(z^2) = 1.84 per pool; pools of one run share packets, so allow 35 %
    assert chi2 < 1.35 * nu / (nu - 2), chi2
    # P(|t_15| > 4) = 1.2e-3
    assert tail <= max(3, 0.005 * len(z)), tail


def test_second_run_equals_a_fresh_run():
    """zero_tallies, stellar emission, self-absorption and dust emission run twice on one engine: the second
    run equals a fresh one (no dust Labs of the first run's last cycle feed the second run's first cycle)."""
    name = "pan_oct_sa"
    sim = S.Simulation(ski(name), packages=1000)
    sim.attach(0)
    for _ in range(2):
        sim.zero_tallies()
        sim.run_stellar()
        sim.run_dust()
        sim.fetch()
    fresh = run_gpu(name, packages=1000, dust=True)
    np.testing.assert_allclose(sim.selfabs_totals(), fresh.selfabs_totals(), rtol=1e-10)
    np.testing.assert_allclose(sim.labs(), fresh.labs(), rtol=1e-10, atol=1e-300)
    np.testing.assert_allclose(sim.labs_dust().sum(axis=0), fresh.labs_dust().sum(axis=0), rtol=1e-10)
    fa, sa = sim.instrument(0)
    fb, sb = fresh.instrument(0)
    np.testing.assert_allclose(sa, sb, rtol=1e-10, atol=1e-300)
    np.testing.assert_allclose(fa.sum(axis=2), fb.sum(axis=2), rtol=1e-10, atol=1e-300)


def _assert_equal_runs(sim, fresh):
    np.testing.assert_allclose(sim.selfabs_totals(), fresh.selfabs_totals(), rtol=1e-10)
    np.testing.assert_allclose(sim.labs(), fresh.labs(), rtol=1e-10, atol=1e-300)
    np.testing.assert_allclose(sim.labs_dust(), fresh.labs_dust(), rtol=1e-10, atol=1e-300)
    fa, sa = sim.instrument(0)
    fb, sb = fresh.instrument(0)
    np.testing.assert_allclose(sa, sb, rtol=1e-10, atol=1e-300)
    np.testing.assert_allclose(fa, fb, rtol=1e-10, atol=1e-300)


def test_a_failed_phase_leaves_no_adds_behind(monkeypatch):
    """A phase that fails after its first trace launches (here the iteration cap, SKIRT_AMD_MAX_ITERATIONS=2,
    'photon phase did not terminate') has added into the Labs replicas, which only the phase-end fold used to
    zero. The next storing phase clears them first: zero_tallies and a good run on the same
    engine equal a fresh engine's run."""
    name = "pan_oct_sa"
    sim = S.Simulation(ski(name), packages=1000)
    sim.attach(0)
    monkeypatch.setenv("SKIRT_AMD_MAX_ITERATIONS", "2")
    with pytest.raises(S.SkirtError, match="did not terminate"):
        sim.run_stellar()
        sim.fetch()
    monkeypatch.delenv("SKIRT_AMD_MAX_ITERATIONS")
    sim.zero_tallies()
    sim.run_stellar()
    sim.run_dust()
    sim.fetch()
    _assert_equal_runs(sim, run_gpu(name, packages=1000, dust=True))


def test_dust_labs_bound_after_a_stellar_phase():
    """Binding caller memory for the dust Labs after a stellar phase that added into Labs replicas (ADVICE r5,
    high): the replicas survive the binding (they used to be freed and then reused and freed again), and the
    self-absorption cycles and dust emission equal a fresh engine's."""
    import torch

    name = "pan_oct_sa"
    sim = S.Simulation(ski(name), packages=1000)
    sim.attach(0)
    sim.run_stellar()
    n_labs, _ = sim.tally_sizes()
    dust = torch.zeros(n_labs, dtype=torch.float64, device="cuda:0")
    sim.bind_dust_labs(dust.data_ptr())
    sim.run_dust()
    sim.fetch()
    assert float(dust.sum()) > 0  # the cycles added into the bound memory
    _assert_equal_runs(sim, run_gpu(name, packages=1000, dust=True))
    del sim
    torch.cuda.synchronize()


def test_transparent_flux_is_deterministic():
    """F_trav = L/(4 pi d^2) for any seed (invariant 4): 2.41996378e-12 W/m2."""
    sim = run_gpu("c1_oligo16", packages=30000, seed=5)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        sim.write(os.path.join(d, "t"))
        sed = F.read_text_tokens(os.path.join(d, "t_i30_sed.dat"))
    assert sed[0][6] == "2.41996378e-12"


@pytest.mark.parametrize("copies", [None, "1", "0"])
def test_many_wavelengths_match_oracle_same_streams(copies, monkeypatch):
    """200 wavelengths and a FullInstrument with 2 scattering levels: 7 slots x 200 SED sums, 8 LDS copies
    of 11.2 KB each (beyond the 64 KB the round-1 engine refused), and the dust phases' device cell
    sources over 200 wavelengths. Also with the detect kernel's SED copies capped at 1, and at 0 (SED adds
    straight to the tally, the fallback when not even one copy fits). Same streams as the oracle."""
    if copies is not None:
        monkeypatch.setenv("SKIRT_AMD_DET_COPIES", copies)
    name = "pan_cart16_l200"
    sim = S.Simulation(ski(name))
    sim.attach(0)
    sim.run_stellar()
    sim.run_dust()
    sim.fetch()
    orc = O.run(ski(name), rng=O.RNG_PHILOX, threads=16, phases=O.PHASES_ALL)
    assert sim.info.nlambda == 200
    np.testing.assert_allclose(sim.labs().sum(axis=0), orc.labs.sum(axis=0), rtol=1e-9)
    assert_parity(sim.labs(), orc.labs, 1e-9, STELLAR_OUTLIERS, "labs")
    frames, seds = sim.instrument(0)
    assert seds.shape == (7, 200) and seds[3:5].sum() > 0 and seds[5:7].sum() > 0
    np.testing.assert_allclose(seds, orc.seds[0], rtol=1e-8, atol=1e-300)
    np.testing.assert_allclose(frames.sum(axis=2), orc.frames[0].sum(axis=2), rtol=1e-8, atol=1e-300)
    assert_parity(frames, orc.frames[0], 1e-8, DUST_OUTLIERS, "frames")


BENCH = os.path.join(os.path.dirname(GOLD), "..", "benchmarks")


@pytest.mark.parametrize("config,packages,labs_global", [("c2_cart64", 20000, "0"), ("c3_oct128", 20000, "0"),
                                                         ("c3_oct128", 20000, "1"), ("c4_vor1e5", 20000, "0"),
                                                         ("c5_oct128_sa", 2000, "0")])
def test_benchmark_models_match_oracle_same_streams(config, packages, labs_global, monkeypatch):
    """The BASELINE configurations at their full grid sizes (C2 64^3 Cartesian, C3 622,490-leaf octree, C4
    1e5-site Voronoi, C5 = C3 with self-absorption and dust emission), at 2e4 packages per wavelength (2e3
    for C5, all of its phases): 5e5 C3 packets, whose paths reach the tree walk's rare branches (the on-face
    neighbour search, the nextafter escape of TreeDustGrid.cpp:502-519) and the Voronoi walk's exact
    re-evaluation. Engine = oracle on the same Philox streams; C3 also with the Labs adds as global atomics
    (SKIRT_AMD_LABS_GLOBAL=1: the path of a Labs table of 4 GiB or more, which no buffer descriptor spans)."""
    monkeypatch.setenv("SKIRT_AMD_LABS_GLOBAL", labs_global)
    path = os.path.join(BENCH, config + ".ski")
    sim = S.Simulation(path, packages=packages)
    sim.attach(0)
    sim.run_stellar()
    sim.run_dust()
    sim.fetch()
    orc = O.run(path, rng=O.RNG_PHILOX, threads=16, packages=packages, phases=O.PHASES_ALL)
    dust = orc.labs_dust is not None or config == "c5_oct128_sa"
    rtol = 1e-8 if dust else 1e-9
    np.testing.assert_allclose(sim.labs().sum(axis=0), orc.labs.sum(axis=0), rtol=1e-9)
    assert_parity(sim.labs(), orc.labs, 1e-9, STELLAR_OUTLIERS, "labs")
    if orc.labs_dust is not None:
        np.testing.assert_allclose(sim.selfabs_totals(), orc.labs_dust_totals, rtol=1e-8)
        assert_parity(sim.labs_dust(), orc.labs_dust, 1e-8, DUST_OUTLIERS, "labs_dust")
    frames, seds = sim.instrument(0)
    np.testing.assert_allclose(seds, orc.seds[0], rtol=rtol, atol=1e-300)
    np.testing.assert_allclose(frames.sum(axis=2), orc.frames[0].sum(axis=2), rtol=rtol, atol=1e-300)
    assert_parity(frames, orc.frames[0], rtol, DUST_OUTLIERS if dust else STELLAR_OUTLIERS, "frames")


@pytest.mark.parametrize("config", ["c3_oct128", "c4_vor1e5"])
def test_full_size_phase_properties(config):
    """The benchmark workload at its full per-GPU size (5e6 packages per wavelength, >= 1e8 packets, the
    2^24-slot pool and its ray queues under full pressure), checked through properties that hold at any
    size: (1) the transparent flux is the emitted luminosity exactly (every launched packet is detected
    once at its full weight: L_lambda / (4 pi d^2) per wavelength, FullInstrument.cpp:115); (2) two
    halves of every wavelength's packets (the reference's IdenticalAssigner split over two ranks, shot
    in their own phases with their own slot schedules) add up to the whole phase cell for cell, pixel for
    pixel, to the order of the atomic additions."""
    path = os.path.join(BENCH, config + ".ski")
    packages = 5e6

    def shoot(rank=None):
        sim = S.Simulation(path, packages=packages)
        sim.attach(0)
        if rank is None:
            sim.run_stellar()
        else:
            sim.set_reducer(lambda tally, ptr, n, stream: None)  # one process: the caller sums
            sim.run_stellar_shard(rank, 2)
        sim.fetch()
        return sim

    full = shoot()
    st = full.stats()
    assert st["packets"] >= 1e8
    # the emitted luminosity per wavelength: the transparent tally of one packet per wavelength (one stellar
    # component: every packet carries L_lambda / Npp, FullInstrument.cpp:115 adds it unattenuated)
    lum = O.run(path, rng=O.RNG_PHILOX, threads=1, packages=1).seds[0][0]
    trav = full.instrument(0)[1][0]  # FullInstrument slot 0 (transparent), before calibration
    assert np.count_nonzero(lum) >= 20
    np.testing.assert_allclose(trav, lum, rtol=1e-10, atol=0)
    halves = [shoot(r) for r in (0, 1)]
    np.testing.assert_allclose(halves[0].labs() + halves[1].labs(), full.labs(), rtol=1e-10, atol=1e-300)
    for k in (0, 1):
        np.testing.assert_allclose(halves[0].instrument(0)[k] + halves[1].instrument(0)[k], full.instrument(0)[k],
                                   rtol=1e-10, atol=1e-300)


def test_continuous_scattering_with_several_instruments(tmp_path):
    """Continuous scattering queues kPathCap peel-offs per instrument and slot, so the slot pool shrinks with
    the instrument count. pan_oct_cs with a FullInstrument, an SEDInstrument and a
    FrameInstrument whose field leaves part of the grid outside (its peel-offs from there are skipped):
    all phases, every instrument against the oracle on the same streams."""
    text = open(ski("pan_oct_cs")).read()
    full = text.index("<FullInstrument")
    end = text.index("/>", full) + 2
    extra = ('\n            <SEDInstrument instrumentName="i0" distance="10 Mpc" inclination="0 deg" azimuth="0 deg"/>'
             '\n            <FrameInstrument instrumentName="f60" distance="10 Mpc" inclination="60 deg" azimuth="-30 deg"'
             ' positionAngle="0 deg" fieldOfViewX="400 pc" pixelsX="16" centerX="50 pc" fieldOfViewY="400 pc"'
             ' pixelsY="16" centerY="0 pc"/>')
    path = os.path.join(tmp_path, "pan_oct_cs3.ski")
    with open(path, "w") as f:
        f.write(text[:end] + extra + text[end:])
    packages = 200
    sim = S.Simulation(path, packages=packages)
    assert sim.info.ninstruments == 3
    sim.attach(0)
    sim.run_stellar()
    sim.run_dust()
    sim.fetch()
    orc = O.run(path, rng=O.RNG_PHILOX, threads=16, packages=packages, phases=O.PHASES_ALL)
    assert_parity(sim.labs(), orc.labs, 1e-9, STELLAR_OUTLIERS, "labs")
    for i in range(3):
        frames, seds = sim.instrument(i)
        assert (seds is None) == (orc.seds[i] is None) and (frames is None) == (orc.frames[i] is None)
        if seds is not None:  # (a FrameInstrument has no SED)
            assert seds.sum() > 0
            np.testing.assert_allclose(seds, orc.seds[i], rtol=1e-8, atol=1e-300)
        if frames is not None:  # (an SEDInstrument has no frame)
            assert frames.sum() > 0
            assert_parity(frames, orc.frames[i], 1e-8, DUST_OUTLIERS, "frames_%d" % i)
