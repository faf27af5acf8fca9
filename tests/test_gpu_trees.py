"""Tree grids on the GPU (k-d trees, barycentric octrees, the TopDown search) against the CPU oracle on
the same Philox streams, and the k-d tree's leaf-map walk against its node-array walk. The variants are
built by tests/tree_models.py from the pinned pan_oct / c1_oligo16 models."""
import numpy as np
import pytest

import oracle_lib as O
import skirt_amd as S
import tree_models as T
from parity import DUST_OUTLIERS, STELLAR_OUTLIERS, assert_parity

pytestmark = pytest.mark.gpu


def run_gpu(path, packages):
    sim = S.Simulation(path, packages=packages)
    sim.attach(0)
    sim.run_stellar()
    sim.fetch()
    return sim


@pytest.mark.parametrize("name,walk", [("bin_pan", S.WALK_KDTREE_MAP), ("bin_pan_td", S.WALK_KDTREE_MAP),
                                       ("bin_full", S.WALK_KDTREE_MAP), ("bin_bary", None),
                                       ("oct_bary", S.WALK_TREE_NODES), ("oct_pan_td", S.WALK_OCTREE_MAP),
                                       ("oct_pan_bk", S.WALK_OCTREE_BOOKKEEPING),
                                       ("oct_bary_bk", S.WALK_OCTREE_BOOKKEEPING)])
def test_tree_engine_matches_oracle_same_streams(tmp_path, name, walk):
    path = T.write(name, str(tmp_path))
    packages = 2000
    sim = run_gpu(path, packages)
    st = sim.stats()
    if walk is not None:
        assert st["grid_walk"] == walk, st
    orc = O.run(path, rng=O.RNG_PHILOX, threads=16, packages=packages)
    assert st["packets"] == orc.packets
    if orc.labs is not None:
        labs = sim.labs()
        np.testing.assert_allclose(labs.sum(), orc.labs.sum(), rtol=1e-9)
        np.testing.assert_allclose(labs.sum(axis=0), orc.labs.sum(axis=0), rtol=1e-9)
        assert_parity(labs, orc.labs, 1e-9, STELLAR_OUTLIERS, "labs")
    frames, seds = sim.instrument(0)
    np.testing.assert_allclose(seds, orc.seds[0], rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(frames.sum(axis=2), orc.frames[0].sum(axis=2), rtol=1e-9, atol=1e-300)
    assert_parity(frames, orc.frames[0], 1e-9, STELLAR_OUTLIERS, "frames")


@pytest.mark.parametrize("name", ["bin_pan", "bin_full"])
def test_kd_tree_leaf_map_walk_equals_node_walk(tmp_path, name, monkeypatch):
    """The k-d tree's leaf map (per-axis leaf extents) takes exactly the node-array walk's steps."""
    path = T.write(name, str(tmp_path))
    runs = []
    for leafmap in ("1", "0"):
        monkeypatch.setenv("SKIRT_AMD_LEAFMAP", leafmap)
        runs.append(run_gpu(path, 2000))
    a, b = runs
    sa, sb = a.stats(), b.stats()
    assert sa["grid_walk"] == S.WALK_KDTREE_MAP and sb["grid_walk"] == S.WALK_TREE_NODES
    for k in ("packets", "segments_fill", "segments_walk", "segments_peel", "detects", "absorb_adds"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])
    if a.labs() is not None:
        np.testing.assert_allclose(a.labs(), b.labs(), rtol=1e-10, atol=1e-300)
    fa, da = a.instrument(0)
    fb, db = b.instrument(0)
    np.testing.assert_allclose(da, db, rtol=1e-10, atol=1e-300)
    np.testing.assert_allclose(fa, fb, rtol=1e-10, atol=1e-300)

