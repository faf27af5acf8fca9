"""Device cell numbering and Cartesian meshes on the GPU.

* Cartesian grids with odd bin counts (2x2x2 device-cell bricks with unused cells) and power-law meshes
  against the CPU oracle on the same Philox streams.
* The line-aligned device numbering (octree sibling leaves and Cartesian bricks on one 64-byte Labs
  line) against the plain numbering (SKIRT_AMD_CELL_ALIGN=0): the same walks
  (identical segment, absorption and detection counts) and the same tallies up to the order of the
  atomic additions."""
import os

import numpy as np
import pytest

import oracle_lib as O
import skirt_amd as S
import tree_models as T
from parity import DUST_OUTLIERS, STELLAR_OUTLIERS, assert_parity, cartesian_neighbour_scale

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ski")


def run_gpu(path, packages):
    sim = S.Simulation(path, packages=packages)
    sim.attach(0)
    sim.run_stellar()
    sim.fetch()
    return sim


@pytest.mark.parametrize("name", ["cart_odd", "cart_pow"])
def test_cartesian_engine_matches_oracle_same_streams(tmp_path, name):
    path = T.write(name, str(tmp_path))
    packages = 3000
    sim = run_gpu(path, packages)
    st = sim.stats()
    assert st["grid_walk"] == S.WALK_CARTESIAN
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


@pytest.mark.parametrize("name", ["cart_odd", "pan_oct"])
def test_aligned_cell_numbering_equals_plain_numbering(tmp_path, name, monkeypatch):
    path = os.path.join(GOLD, name + ".ski") if name == "pan_oct" else T.write(name, str(tmp_path))
    runs = []
    for align in ("1", "0"):
        monkeypatch.setenv("SKIRT_AMD_CELL_ALIGN", align)
        runs.append(run_gpu(path, 3000))
    a, b = runs
    sa, sb = a.stats(), b.stats()
    assert sa["device_cells"] > sb["device_cells"] == a.info.ncells  # aligned: unused device cells
    for k in ("packets", "segments_fill", "segments_walk", "segments_peel", "detects", "absorb_adds"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    assert sa["labs_requests"] < sb["labs_requests"]  # the point of the alignment
    np.testing.assert_allclose(a.labs(), b.labs(), rtol=1e-12, atol=1e-300)
    fa, da = a.instrument(0)
    fb, db = b.instrument(0)
    np.testing.assert_allclose(da, db, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(fa, fb, rtol=1e-12, atol=1e-300)


def test_labs_table_over_4_gib_takes_global_atomics(tmp_path):
    """A Labs table of more than 4 GiB (128^3 cells x 257 wavelengths x 8 B = 4.31e9 B), beyond what the trace
    kernel's buffer descriptor spans: the drain adds with global atomics instead, and the
    engine equals the oracle on the same streams."""
    text = open(os.path.join(GOLD, "pan_cart16.ski")).read()
    for n in ("X", "Y", "Z"):
        old = '<mesh%s type="MoveableMesh"><LinMesh numBins="16"/></mesh%s>' % (n, n)
        assert text.count(old) == 1
        text = text.replace(old, '<mesh%s type="MoveableMesh"><LinMesh numBins="128"/></mesh%s>' % (n, n))
    assert text.count('points="10"') == 1
    text = text.replace('points="10"', 'points="257"')
    path = os.path.join(str(tmp_path), "cart_big.ski")
    with open(path, "w") as f:
        f.write(text)
    packages = 20
    sim = run_gpu(path, packages)
    assert sim.info.ncells == 128 ** 3 and sim.info.nlambda == 257
    assert sim.stats()["device_cells"] * 257 * 8 > 2 ** 32
    orc = O.run(path, rng=O.RNG_PHILOX, threads=16, packages=packages)
    assert sim.stats()["packets"] == orc.packets
    labs = sim.labs()
    assert labs.sum() > 0
    np.testing.assert_allclose(labs.sum(axis=0), orc.labs.sum(axis=0), rtol=1e-9, atol=1e-300)
    # Round 5 ran this at 1e-8: 28 of 960,185 elements were beyond 1e-9, the largest 1.34e-7 (cell 317912,
    # wavelength 44), profiles/r05_labs_over_4gib.txt. The packet trace (profiles/r06_parity_trace.txt,
    # tools/parity_trace.py) found no changed decision: packet 890 alone adds to that cell, engine and oracle
    # cross the same 115 cells of its third FILL path, and the cell is a sliver of it, 1.2e11 m against a
    # median segment of 1.6e17 m. The path starts 1 ulp apart in position and 1-3 ulp in direction (the
    # engine's equivalent scattering formulas), every segment agrees to 1.6e-13 of the
    # median segment, and the sliver's length -- the difference of two coordinates equal to 7e-7 of a cell --
    # carries that as 1.3e-7 of itself. So the comparison is at 1e-9 with no outlier again, the slivers
    # judged against their neighbours' full crossings (parity.cartesian_neighbour_scale). The global atomics
    # play no part: at 200 wavelengths (3.4 GB, the buffer descriptor's path) SKIRT_AMD_LABS_GLOBAL=0 and =1
    # give bit-identical tallies (profiles/r05_labs_over_4gib.txt).
    assert_parity(labs, orc.labs, 1e-9, STELLAR_OUTLIERS, "labs",
                  slivers=cartesian_neighbour_scale(orc.labs, (128, 128, 128)))
    del labs, orc


def _cart_model(tmp_path, bins, points, name, max_wavelength=None):
    text = open(os.path.join(GOLD, "pan_cart16.ski")).read()
    if max_wavelength:
        assert text.count('maxWavelength="1000 micron"') == 1
        text = text.replace('maxWavelength="1000 micron"', 'maxWavelength="%s"' % max_wavelength)
    for n in ("X", "Y", "Z"):
        old = '<mesh%s type="MoveableMesh"><LinMesh numBins="16"/></mesh%s>' % (n, n)
        assert text.count(old) == 1
        text = text.replace(old, '<mesh%s type="MoveableMesh"><LinMesh numBins="%d"/></mesh%s>' % (n, bins, n))
    assert text.count('points="10"') == 1
    text = text.replace('points="10"', 'points="%d"' % points)
    path = os.path.join(str(tmp_path), name)
    with open(path, "w") as f:
        f.write(text)
    return path


def test_labs_high_index_bits_equal_the_32_bit_indices(tmp_path, monkeypatch):
    """The buffered Labs adds of a table of 2^32 elements or more carry bits 32-39 of the element index in a
    byte of their own (Args::labsHi); SKIRT_AMD_LABS_HI=1 forces that path on a small table: the same
    packets, the same tallies as the 32-bit global-atomics path, up to the order of the additions."""
    path = _cart_model(tmp_path, 64, 10, "cart64.ski")
    runs = []
    for env in ("SKIRT_AMD_LABS_GLOBAL", "SKIRT_AMD_LABS_HI"):
        monkeypatch.delenv("SKIRT_AMD_LABS_GLOBAL", raising=False)
        monkeypatch.delenv("SKIRT_AMD_LABS_HI", raising=False)
        monkeypatch.setenv(env, "1")
        runs.append(run_gpu(path, 2000))
    a, b = runs
    for k in ("packets", "segments_fill", "segments_walk", "segments_peel", "detects", "absorb_adds"):
        assert a.stats()[k] == b.stats()[k], k
    assert a.labs().sum() > 0
    np.testing.assert_allclose(a.labs(), b.labs(), rtol=1e-12, atol=1e-300)


@pytest.mark.timeout(600)
def test_labs_table_of_2_32_elements_or_more(tmp_path):
    """A Labs table of more than 2^32 elements (256^3 cells x 280 wavelengths = 4.70e9 doubles, 37.6 GB),
    which round 5 refused (VERDICT r5 missing 4; the reference's ArrayTable has no such limit,
    Fundamentals/Table.hpp:104-105): the adds carry 40-bit element indices. Against the oracle on the same
    streams: the per-wavelength totals, and every element of the 24 wavelengths whose rows lie past 2^32
    elements (a lost high byte would put their adds 32 GiB lower). The wavelengths end at 20 micron, so
    that every one of them carries stellar luminosity. The tallies stay on the device (bound tensors) and
    are checked there: no 37.6 GB download."""
    import torch

    nl = 280
    path = _cart_model(tmp_path, 256, nl, "cart256.ski", max_wavelength="20 micron")
    packages = 20
    sim = S.Simulation(path, packages=packages)
    assert sim.info.ncells == 256 ** 3 and sim.info.nlambda == nl
    sim.attach(0)
    n_labs, n_instr = sim.tally_sizes()
    assert n_labs > 2 ** 32
    labs = torch.zeros(n_labs, dtype=torch.float64, device="cuda:0")
    instr = torch.zeros(n_instr, dtype=torch.float64, device="cuda:0")
    sim.bind_tallies(labs.data_ptr(), instr.data_ptr())
    sim.zero_tallies()
    sim.run_stellar()
    sim.synchronize()
    stride = n_labs // nl
    first = -(-2 ** 32 // stride)  # the first wavelength whose row starts at 2^32 elements or beyond
    assert first < nl
    rows = labs.view(nl, stride)
    sums = rows.sum(dim=1).cpu().numpy()
    # the reference cell order of those rows: the engine's bricked Cartesian numbering
    # (Grid<SKIRT_GRID_CARTESIAN>::dev), cell m = k + n j + n^2 i
    n = 256
    m = torch.arange(n ** 3, device="cuda:0", dtype=torch.int64)
    i, j, k = m // (n * n), (m // n) % n, m % n
    b = n // 2
    dev = ((((i >> 1) * b + (j >> 1)) * b + (k >> 1)) << 3) | ((i & 1) << 2) | ((j & 1) << 1) | (k & 1)
    high = rows[first:][:, dev].t().contiguous().cpu().numpy()  # cells x the high wavelengths
    del labs, rows, m, i, j, k, dev
    torch.cuda.empty_cache()
    orc = O.run(path, rng=O.RNG_PHILOX, threads=16, packages=packages)
    assert sim.stats()["packets"] == orc.packets
    ref_sums = orc.labs.sum(axis=0)
    ref_high = np.ascontiguousarray(orc.labs[:, first:])
    del orc
    assert np.all(ref_sums > 0) and np.all(ref_high.sum(axis=0) > 0)
    np.testing.assert_allclose(sums, ref_sums, rtol=1e-9, atol=1e-300)
    assert_parity(high, ref_high, 1e-9, STELLAR_OUTLIERS, "labs past 2^32 elements",
                  slivers=cartesian_neighbour_scale(ref_high, (n, n, n)))
