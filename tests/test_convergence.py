"""DustSystem::writeconvergence (DustSystem.cpp:195-305) in the oracle: <prefix>_ds_convergence.dat holds the
grid's mass and its column densities through the origin beside the dust distribution's analytic values.
The reference's fixtures all set writeConvergence="false", so there is no reference file to compare with
(pinned against the reference by the pan_oct_out, pan_cart16_out and vor_pan_out fixtures); these checks also pin the format and the physics: the grid's values
approach the analytic ones, spherical models write the radial branch, an exponential disk the edge-on and
face-on branches. tests/test_gpu_counts.py compares the engine's file with the oracle's."""
import os

import pytest

import oracle_lib as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "ski")


def convergence_ski(tmp_path, name, disk=False):
    text = open(os.path.join(GOLD, name + ".ski")).read().replace('writeConvergence="false"', 'writeConvergence="true"')
    if disk:  # the dust component's geometry (the second Plummer geometry of the file) as an exponential disk
        plummer = '<PlummerGeometry scale="100 pc"/>'
        i = text.index(plummer, text.index(plummer) + 1)
        text = text[:i] + '<ExpDiskGeometry radialScale="100 pc" axialScale="20 pc"/>' + text[i + len(plummer):]
    path = os.path.join(tmp_path, name + ("_disk" if disk else "") + ".ski")
    with open(path, "w") as f:
        f.write(text)
    return path


def values(text):
    """(quantity, expected, actual) triples of a convergence file"""
    lines = text.splitlines()
    out = []
    for i, l in enumerate(lines):
        if l.startswith("   - "):
            e = float(lines[i + 1].split("=")[1].split()[0])
            a = float(lines[i + 2].split("=")[1].split()[0])
            out.append((l[5:], e, a))
    return out


@pytest.mark.parametrize("name,disk", [("pan_cart16", False), ("pan_oct", False), ("vor_pan", False),
                                       ("oligo_2comp", False), ("pan_oct", True)],
                         ids=["cart", "oct", "vor", "oligo_2comp", "oct_disk"])
def test_oracle_convergence_file(tmp_path, name, disk):
    ski = convergence_ski(tmp_path, name, disk)
    O.run(ski, rng=O.RNG_PHILOX, threads=4, packages=10, phases=O.PHASES_STELLAR, outprefix=os.path.join(tmp_path, "o"))
    text = open(os.path.join(tmp_path, "o_ds_convergence.dat")).read()
    assert text.startswith("Convergence check on the grid: \n")
    v = values(text)
    names = [q for q, _, _ in v]
    if disk:
        assert names == ["edge-on (R-axis) surface density", "face-on (Z-axis) surface density", "total dust mass"]
    else:
        assert names == ["radial (r-axis) surface density", "total dust mass"]
    for q, e, a in v:
        assert e > 0 and a > 0
        # a 16^3 grid through the origin of a cusp-free profile: within tens of percent of the analytic value
        assert abs(a / e - 1) < 0.5, (q, e, a)
    assert " Msun/pc2\n" in text and text.rstrip().endswith("Msun")
