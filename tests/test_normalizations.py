"""Dust component normalizations by optical depth (FaceOnDustCompNormalization,
EdgeOnDustCompNormalization, RadialDustCompNormalization: tau / (Sigma * kappaext(lambda)) with
AxGeometry::SigmaZ / SigmaR or SpheGeometry::Sigmar, DustMix::kappaext's log-log interpolation).
Restated here from the reference formulas; the faceon_cart, edgeon_cart and radial_cart reference fixtures pin
them too (tests/test_oracle_golden.py)."""
import math

import numpy as np
import pytest

import oracle_lib as O
import tree_models as T
from test_geometries import PC

NORMS = {
    "faceon": '<FaceOnDustCompNormalization wavelength="0.55 micron" opticalDepth="0.7"/>',
    "edgeon": '<EdgeOnDustCompNormalization wavelength="1.3 micron" opticalDepth="4"/>',
    "radial": '<RadialDustCompNormalization wavelength="0.55 micron" opticalDepth="2.5"/>',
}


def kappaext(kext, lam, x):
    ell = np.searchsorted(lam, x, side="right") - 1
    p = (math.log10(x) - math.log10(lam[ell])) / (math.log10(lam[ell + 1]) - math.log10(lam[ell]))
    kL, kR = kext[ell], kext[ell + 1]
    lL, lR = math.log10(kL), math.log10(kR)
    return math.pow(10, lL + p * (lR - lL))


@pytest.mark.parametrize("norm", ["faceon", "edgeon", "radial"])
def test_optical_depth_normalizations(tmp_path, norm):
    # disk dust for the axisymmetric ones, the model's Plummer dust for the radial one
    if norm == "faceon":  # a disk without inner radius (SigmaZ = 0 for Rmin > 0, ExpDiskGeometry::SigmaZ)
        T.GEOMETRIES["_probe"] = ("pan_cart16", T.STAR_DISK, T.STAR_DISK)
        try:
            path = T.write_geometry("_probe", str(tmp_path))
        finally:
            del T.GEOMETRIES["_probe"]
    elif norm == "edgeon":
        path = T.write_geometry("disk_cart", str(tmp_path))
    else:
        path = str(tmp_path / "plummer.ski")
        with open(path, "w") as f:
            f.write(open(T.os.path.join(T.GOLD, "pan_cart16.ski")).read())
    text = open(path).read()
    old = text[text.index("<DustMassDustCompNormalization"):]
    old = old[:old.index("/>") + 2]
    with open(path, "w") as f:
        f.write(text.replace(old, NORMS[norm]))
    nf, kext, lam = O.dust_component(path)
    if norm == "faceon":  # ExpDisk {hR 120, hz 25} pc, no truncation: SigmaZ = 2 rho0 hz = 1 / (2 pi hR^2)
        hR, hz = 120 * PC, 25 * PC
        rho0 = 1.0 / (hR * hR * 1.0 * 2 * math.pi * (2.0 * hz))
        Sigma = 2.0 * rho0 * hz
        tau, x = 0.7, 0.55e-6
    elif norm == "edgeon":
        hR, hz, Rmax, zmax, Rmin = 150 * PC, 40 * PC, 450 * PC, 300 * PC, 20 * PC
        intz = -2 * hz * math.expm1(-zmax / hz)
        tmin = math.exp(-Rmin / hR) * (1 + Rmin / hR)
        tmax = math.exp(-Rmax / hR) * (1 + Rmax / hR)
        rho0 = 1.0 / (hR * hR * (tmin - tmax) * 2 * math.pi * intz)
        Sigma = rho0 * hR * (math.exp(-Rmin / hR) - math.exp(-Rmax / hR))
        tau, x = 4.0, 1.3e-6
    else:
        c = 100 * PC
        Sigma = 0.5 / (math.pi * c * c)
        tau, x = 2.5, 0.55e-6
    np.testing.assert_allclose(nf, tau / (Sigma * kappaext(kext, lam, x)), rtol=1e-12)
