"""The oracle's path statistics on the CPU: its segment counts add up (FILL paths + peel-off paths = all
paths it built), and its cells-crossed histogram (DustSystem's _crossed, DustSystem.cpp:959-1000) holds every
path once; the ds_crossed file follows DustSystem::write (DustSystem.cpp:1004-1024) and TextOutFile's 'd'
columns. The engine's device counters are compared with these on the GPU (test_gpu_counts.py)."""
import os

import numpy as np

import oracle_lib as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ski")


def test_oracle_counts_add_up():
    orc = O.run(os.path.join(GOLD, "pan_oct.ski"), rng=O.RNG_PHILOX, threads=4, packages=300)
    assert orc.segments == orc.segments_fill + orc.segments_peel
    n = np.arange(len(orc.crossed), dtype=np.uint64)
    assert int((orc.crossed * n).sum()) == orc.segments
    assert 0 < orc.absorb_adds <= orc.segments_fill
    # one peel-off path per launch and scattering (one instrument), at least one FILL path per launch
    assert int(orc.crossed.sum()) >= 2 * orc.packets


def test_oracle_counts_do_not_depend_on_threads():
    a = O.run(os.path.join(GOLD, "vor_pan.ski"), rng=O.RNG_PHILOX, threads=1, packages=100)
    b = O.run(os.path.join(GOLD, "vor_pan.ski"), rng=O.RNG_PHILOX, threads=8, packages=100)
    assert (a.segments_fill, a.segments_peel, a.absorb_adds) == (b.segments_fill, b.segments_peel, b.absorb_adds)
    np.testing.assert_array_equal(a.crossed, b.crossed)


def test_ds_crossed_file_format(tmp_path):
    text = open(os.path.join(GOLD, "pan_cart16.ski")).read().replace('writeCellsCrossed="false"',
                                                                     'writeCellsCrossed="true"')
    path = os.path.join(tmp_path, "m.ski")
    with open(path, "w") as f:
        f.write(text)
    orc = O.run(path, rng=O.RNG_MT, packages=200, outprefix=os.path.join(tmp_path, "o"))
    lines = open(os.path.join(tmp_path, "o_ds_crossed.dat")).read().splitlines()
    assert lines[0] == "# total number of cells in grid: 4096"
    assert lines[1] == "# column 1: number of cells crossed"
    assert lines[2] == "# column 2: number of paths that crossed this number of cells"
    rows = [tuple(int(v) for v in l.split()) for l in lines[3:]]
    assert [r[0] for r in rows] == list(range(len(rows)))
    assert [r[1] for r in rows] == [int(v) for v in orc.crossed]
    assert rows[-1][1] > 0
