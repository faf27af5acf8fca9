"""MeanZubkoDustMix and DraineLiDustMix (MeanZubkoDustMix.cpp, DraineLiDustMix.cpp, DustMix::addpopulation):
the packaged tables (skirt_amd/data/*.bin, written by tools/convert_dat.py) hold the reference's data
files' numbers, and models using the mixes run. No reference fixture uses these mixes: beyond the data
and the shared DustMix code (pinned through InterstellarDustMix), pinned against the reference by the zubko_cart and draineli_cart fixtures;
the GPU engine matches the oracle on them (tests/test_gpu_geometries.py)."""
import os
import struct

import numpy as np
import pytest

import oracle_lib as O
import tree_models as T

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DAT = "/root/reference/dat/DustMix"


def read_bin(name):
    with open(os.path.join(REPO, "skirt_amd", "data", name), "rb") as f:
        nrows, ncols = struct.unpack("<qq", f.read(16))
        return np.frombuffer(f.read(), dtype="<f8").reshape(nrows, ncols)


@pytest.mark.skipif(not os.path.isdir(REF_DAT), reason="reference data files absent (GPU box)")
@pytest.mark.parametrize("name,n", [("MeanZubkoDustMix", 1201), ("DraineLiDustMix", 800)])
def test_packaged_tables_hold_the_reference_numbers(name, n):
    rows = []
    with open(os.path.join(REF_DAT, name + ".dat")) as f:
        for line in f:
            s = line.strip()
            if s and not s.startswith("#"):
                rows.append([float(t) for t in s.split()])
    np.testing.assert_array_equal(read_bin(name + ".bin"), np.array(rows[:n]))


@pytest.mark.parametrize("name", ["zubko_cart", "draineli_cart"])
def test_mix_models_run(tmp_path, name):
    path = T.write_mix(name, str(tmp_path))
    a = O.run(path, rng=O.RNG_MT, threads=1, packages=300)
    b = O.run(path, rng=O.RNG_MT, threads=1, packages=300)
    np.testing.assert_array_equal(a.labs, b.labs)
    assert np.isfinite(a.labs).all() and a.labs.sum() > 0
    t = read_bin(("MeanZubkoDustMix" if name.startswith("zubko") else "DraineLiDustMix") + ".bin")
    assert np.all(np.diff(t[:, 0]) > 0)  # increasing wavelengths, as addpopulation resamples them
