"""Variants of the golden models (tree grids, Cartesian meshes, geometries, mixes, SEDs, normalizations, diagnostic
outputs), written as .ski files for the tests and for tests/golden/make_fixtures.sh, which runs the rebuilt reference
(oracle/ref.mk) on each to write its reference fixture: BinTreeDustGrid (the k-d tree, Alternating or Barycenter
split directions, BinTreeDustGrid.cpp, BinTreeNode.cpp, BaryBinTreeNode.cpp), barycentric octrees
(BaryOctTreeNode.cpp), the TopDown and Bookkeeping searches, and the others below. Each swaps one element of a
committed model."""
import os
import re

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ski")
BOX = 'minX="-500 pc" maxX="500 pc" minY="-500 pc" maxY="500 pc" minZ="-500 pc" maxZ="500 pc"'

GRIDS = {
    # full trees: every node is split down to maxLevel, so the octree of level 4 and the k-d tree of
    # level 12 have the same 4096 leaf boxes (16^3)
    "oct_full": ("c1_oligo16", '<OctTreeDustGrid writeGrid="false" %s minLevel="1" maxLevel="4" searchMethod="Neighbor" '
                 'sampleCount="10" maxOpticalDepth="0" maxMassFraction="0" maxDensDispFraction="0" barycentric="false"/>'),
    "bin_full": ("c1_oligo16", '<BinTreeDustGrid writeGrid="false" %s minLevel="3" maxLevel="12" searchMethod="Neighbor" '
                 'sampleCount="10" maxOpticalDepth="0" maxMassFraction="0" maxDensDispFraction="0" '
                 'directionMethod="Alternating"/>'),
    "bin_full_td": ("c1_oligo16", '<BinTreeDustGrid writeGrid="false" %s minLevel="3" maxLevel="12" searchMethod="TopDown" '
                    'sampleCount="10" maxOpticalDepth="0" maxMassFraction="0" maxDensDispFraction="0" '
                    'directionMethod="Alternating"/>'),
    # adaptive trees on the Pan model of the pan_oct fixture
    "bin_pan": ("pan_oct", '<BinTreeDustGrid writeGrid="false" %s minLevel="6" maxLevel="18" searchMethod="Neighbor" '
                'sampleCount="100" maxOpticalDepth="0" maxMassFraction="5e-4" maxDensDispFraction="0" '
                'directionMethod="Alternating"/>'),
    "bin_pan_td": ("pan_oct", '<BinTreeDustGrid writeGrid="false" %s minLevel="6" maxLevel="18" searchMethod="TopDown" '
                   'sampleCount="100" maxOpticalDepth="0" maxMassFraction="5e-4" maxDensDispFraction="0" '
                   'directionMethod="Alternating"/>'),
    "bin_bary": ("pan_oct", '<BinTreeDustGrid writeGrid="false" %s minLevel="3" maxLevel="18" searchMethod="Neighbor" '
                 'sampleCount="100" maxOpticalDepth="0" maxMassFraction="5e-4" maxDensDispFraction="0" '
                 'directionMethod="Barycenter"/>'),
    "oct_bary": ("pan_oct", '<OctTreeDustGrid writeGrid="false" %s minLevel="1" maxLevel="6" searchMethod="Neighbor" '
                 'sampleCount="100" maxOpticalDepth="0" maxMassFraction="5e-4" maxDensDispFraction="0" barycentric="true"/>'),
    "oct_pan_td": ("pan_oct", '<OctTreeDustGrid writeGrid="false" %s minLevel="2" maxLevel="6" searchMethod="TopDown" '
                   'sampleCount="100" maxOpticalDepth="0" maxMassFraction="5e-4" maxDensDispFraction="0" barycentric="false"/>'),
    "oct_pan_bk": ("pan_oct", '<OctTreeDustGrid writeGrid="false" %s minLevel="2" maxLevel="6" searchMethod="Bookkeeping" '
                   'sampleCount="100" maxOpticalDepth="0" maxMassFraction="5e-4" maxDensDispFraction="0" barycentric="false"/>'),
    "oct_bary_bk": ("pan_oct", '<OctTreeDustGrid writeGrid="false" %s minLevel="1" maxLevel="6" searchMethod="Bookkeeping" '
                    'sampleCount="100" maxOpticalDepth="0" maxMassFraction="5e-4" maxDensDispFraction="0" barycentric="true"/>'),
    # Cartesian grids on the Pan model of the pan_cart16 fixture: odd bin counts (the engine's 2x2x2
    # device-cell bricks then have unused cells) and the power-law meshes (PowMesh, SymPowMesh with an
    # odd and an even bin count)
    "cart_odd": ("pan_cart16", '<CartesianDustGrid writeGrid="false" %s><meshX type="MoveableMesh"><LinMesh numBins="7"/></meshX>'
                 '<meshY type="MoveableMesh"><LinMesh numBins="5"/></meshY><meshZ type="MoveableMesh"><LinMesh numBins="9"/></meshZ>'
                 '</CartesianDustGrid>'),
    "cart_pow": ("pan_cart16", '<CartesianDustGrid writeGrid="false" %s><meshX type="MoveableMesh"><PowMesh numBins="12" ratio="4"/></meshX>'
                 '<meshY type="MoveableMesh"><SymPowMesh numBins="9" ratio="3"/></meshY>'
                 '<meshZ type="MoveableMesh"><SymPowMesh numBins="10" ratio="0.2"/></meshZ></CartesianDustGrid>'),
}


# ExpDiskGeometry variants: stars and dust in exponential disks (the first PlummerGeometry of a model is
# its stellar component's, the second its dust component's)
STAR_DISK = '<ExpDiskGeometry radialScale="120 pc" axialScale="25 pc" radialTrunc="0 pc" axialTrunc="0 pc" innerRadius="0 pc"/>'
DUST_DISK = ('<ExpDiskGeometry radialScale="150 pc" axialScale="40 pc" radialTrunc="450 pc" axialTrunc="300 pc" '
             'innerRadius="20 pc"/>')
SERSIC4 = '<SersicGeometry index="4" radius="60 pc"/>'
SERSIC1 = '<SersicGeometry index="1.5" radius="120 pc"/>'
POINT = '<PointGeometry/>'
GEOMETRIES = {
    "disk_cart": ("pan_cart16", STAR_DISK, DUST_DISK),
    "disk_oct": ("pan_oct", STAR_DISK, DUST_DISK),
    # a Sersic bulge in a dust disk, and Sersic dust (density sampling of the host setup)
    "bulge_oct": ("pan_oct", SERSIC4, DUST_DISK),
    "sersic_cart": ("pan_cart16", SERSIC1, SERSIC4),
    # a point source (PointGeometry) at the origin, a cell corner of both grids
    "point_oct": ("pan_oct", POINT, DUST_DISK),
    "point_cart": ("pan_cart16", POINT, DUST_DISK),
    # dust in a disk without inner radius (a face-on normalization needs SigmaZ > 0: ExpDiskGeometry::SigmaZ is 0
    # for Rmin > 0)
    "disk0_cart": ("pan_cart16", STAR_DISK, STAR_DISK),
}


def write_geometry(name, directory):
    """Writes geometry variant `name` into `directory` and returns its path."""
    base, star, dust = GEOMETRIES[name]
    text = open(os.path.join(GOLD, base + ".ski")).read()
    parts = text.split('<PlummerGeometry scale="100 pc"/>')
    assert len(parts) == 3, name
    text = parts[0] + star + parts[1] + dust + parts[2]
    path = os.path.join(directory, name + ".ski")
    with open(path, "w") as f:
        f.write(text)
    return path


# dust mixes besides InterstellarDustMix, on the Pan Cartesian model
MIXES = {
    "zubko_cart": ("pan_cart16", '<MeanZubkoDustMix writeMix="false" writeMeanMix="false"/>'),
    "draineli_cart": ("pan_cart16", '<DraineLiDustMix writeMix="false" writeMeanMix="false"/>'),
}


def write_mix(name, directory):
    """Writes dust-mix variant `name` into `directory` and returns its path."""
    base, mix = MIXES[name]
    text = open(os.path.join(GOLD, base + ".ski")).read()
    old = '<InterstellarDustMix writeMix="false" writeMeanMix="false"/>'
    assert text.count(old) == 1, name
    path = os.path.join(directory, name + ".ski")
    with open(path, "w") as f:
        f.write(text.replace(old, mix))
    return path


def write(name, directory):
    """Writes variant `name` into `directory` and returns its path."""
    base, grid = GRIDS[name]
    text = open(os.path.join(GOLD, base + ".ski")).read()
    text, n = re.subn(r'<dustGrid type="DustGrid">.*?</dustGrid>',
                      '<dustGrid type="DustGrid">%s</dustGrid>' % (grid % BOX), text, flags=re.S)
    assert n == 1, name
    path = os.path.join(directory, name + ".ski")
    with open(path, "w") as f:
        f.write(text)
    return path


# the reference's diagnostic outputs switched on: ds_convergence (DustSystem.cpp:195-420), ds_crossed
# (DustSystem.cpp:1004-1024) and ds_cellprops (DustSystem.cpp:636-660)
OUTPUTS = {"pan_oct_out": "pan_oct", "pan_cart16_out": "pan_cart16", "vor_pan_out": "vor_pan"}


def write_outputs(name, directory):
    """Writes output variant `name` into `directory` and returns its path."""
    text = open(os.path.join(GOLD, OUTPUTS[name] + ".ski")).read()
    for attr in ("writeConvergence", "writeCellsCrossed", "writeCellProperties"):
        text, n = re.subn(attr + '="false"', attr + '="true"', text)
        assert n <= 1, (name, attr)
    path = os.path.join(directory, name + ".ski")
    with open(path, "w") as f:
        f.write(text)
    return path


# stellar SEDs besides SunSED, and dust normalizations by optical depth, on the Pan Cartesian model (the
# normalizations on its disk variant, as tests/test_normalizations.py uses them)
SEDS = {"bbody_cart": ("pan_cart16", '<BlackBodySED temperature="20000 K"/>'),
        "quasar_cart": ("pan_cart16", "<QuasarSED/>")}
NORMALIZATIONS = {
    "faceon_cart": ("disk0_cart", '<FaceOnDustCompNormalization wavelength="0.55 micron" opticalDepth="0.7"/>'),
    "edgeon_cart": ("disk_cart", '<EdgeOnDustCompNormalization wavelength="1.3 micron" opticalDepth="4"/>'),
    "radial_cart": ("pan_cart16", '<RadialDustCompNormalization wavelength="0.55 micron" opticalDepth="2.5"/>'),
}


def write_sed(name, directory):
    """Writes SED variant `name` into `directory` and returns its path."""
    base, sed = SEDS[name]
    text = open(os.path.join(GOLD, base + ".ski")).read()
    assert text.count("<SunSED/>") == 1, name
    path = os.path.join(directory, name + ".ski")
    with open(path, "w") as f:
        f.write(text.replace("<SunSED/>", sed))
    return path


def write_normalization(name, directory):
    """Writes dust-normalization variant `name` into `directory` and returns its path."""
    base, norm = NORMALIZATIONS[name]
    src = write_any(base, directory) if base in GEOMETRIES else os.path.join(GOLD, base + ".ski")
    text = open(src).read()
    old = text[text.index("<DustMassDustCompNormalization"):]
    old = old[:old.index("/>") + 2]
    path = os.path.join(directory, name + ".ski")
    with open(path, "w") as f:
        f.write(text.replace(old, norm))
    return path


def write_any(name, directory):
    """Writes the variant `name` of any kind (grid, geometry, mix, outputs, SED, normalization) and returns its
    path."""
    for table, writer in ((GRIDS, write), (GEOMETRIES, write_geometry), (MIXES, write_mix), (OUTPUTS, write_outputs),
                          (SEDS, write_sed), (NORMALIZATIONS, write_normalization)):
        if name in table:
            return writer(name, directory)
    raise KeyError(name)
