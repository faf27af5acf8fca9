"""Stellar SEDs of PanStellarComp besides SunSED: BlackBodySED (BlackBodySED.cpp setupSelfBefore: a
101-point trapezoid of B(lambda) lambda over log lambda per wavelength bin) and QuasarSED (QuasarSED.cpp:
a broken power law in micron, SED::setemissivities), normalized by SED::setluminosities.

A dust-free model makes every packet end at its emission peel-off with weight 1, so the raw SED of an
SEDInstrument at wavelength ell is the sum of the packet luminosities, i.e. the component luminosity
L_ell = Ltot * sed_ell. The restatements below (same formulas, same order, numpy/libm) check the host
tables through the oracle. The bbody_cart and quasar_cart reference fixtures pin them too (tests/test_oracle_golden.py).
"""
import math

import numpy as np
import pytest

import oracle_lib as O

SKI = """<?xml version="1.0" encoding="UTF-8"?>
<skirt-simulation-hierarchy type="MonteCarloSimulation" format="6.1">
    <PanMonteCarloSimulation packages="100" minWeightReduction="1e4" minScattEvents="0" scattBias="0.5" continuousScattering="false">
        <random type="Random"><Random seed="4357"/></random>
        <units type="Units"><ExtragalacticUnits/></units>
        <instrumentSystem type="InstrumentSystem"><InstrumentSystem><instruments type="Instrument">
            <SEDInstrument instrumentName="sed" distance="10 Mpc" inclination="30 deg" azimuth="0 deg"/>
        </instruments></InstrumentSystem></instrumentSystem>
        <wavelengthGrid type="PanWavelengthGrid"><LogWavelengthGrid writeWavelengths="false" minWavelength="0.005 micron" maxWavelength="2000 micron" points="%(N)d"/></wavelengthGrid>
        <stellarSystem type="StellarSystem"><StellarSystem emissionBias="0.5"><components type="StellarComp">
            <PanStellarComp>
                <geometry type="Geometry"><PlummerGeometry scale="100 pc"/></geometry>
                <sed type="StellarSED">%(SED)s</sed>
                <normalization type="StellarCompNormalization"><BolLuminosityStellarCompNormalization luminosity="1e10"/></normalization>
            </PanStellarComp>
        </components></StellarSystem></stellarSystem>
    </PanMonteCarloSimulation>
</skirt-simulation-hierarchy>
"""


def loggrid(lmin, lmax, N):
    n = N - 1
    logxmin = math.log10(lmin)
    dlogx = math.log10(lmax / lmin) / n
    lam = [math.pow(10, logxmin + i * dlogx) for i in range(n + 1)]
    lo = [lam[0]] + [math.sqrt(lam[i - 1] * lam[i]) for i in range(1, N)]
    hi = [math.sqrt(lam[i] * lam[i + 1]) for i in range(N - 1)] + [lam[-1]]
    return lam, lo, hi


def planck(T, lam):
    h, c, k = 6.62606957e-34, 2.99792458e8, 1.3806488e-23
    x = h * c / (lam * k * T)
    e = math.exp(x) if x < 709.78 else math.inf  # C's exp overflows to inf: B = 0
    return 2.0 * h * c * c / math.pow(lam, 5) / (e - 1.0)


def blackbody(T, lo, hi):
    Lv = []
    for a, b in zip(lo, hi):
        N = 100
        l0, l1 = math.log10(a), math.log10(b)
        d = (l1 - l0) / N
        s = 0.0
        for i in range(N + 1):
            w = 0.5 if i in (0, N) else 1.0
            lam = math.pow(10, l0 + i * d)
            s += w * planck(T, lam) * lam
        Lv.append(s * math.log(10) * d)
    return np.array(Lv)


def quasar(lam, lo, hi):
    out = []
    for x, a, b in zip(lam, lo, hi):
        m = x * 1e6
        if m < 0.001: j = 0.0
        elif m < 0.01: j = 1.0 * math.pow(m, 0.2)
        elif m < 0.1: j = 0.003981072 * math.pow(m, -1.0)
        elif m < 5.0: j = 0.001258926 * math.pow(m, -1.5)
        elif m < 1000.0: j = 0.070376103 * math.pow(m, -4.0)
        else: j = 0.0
        out.append(j * (b - a))
    return np.array(out)


@pytest.mark.parametrize("sed", ["bb3000", "bb20000", "quasar"])
def test_stellar_sed_tables(tmp_path, sed):
    N = 25
    xml = {"bb3000": '<BlackBodySED temperature="3000 K"/>', "bb20000": '<BlackBodySED temperature="20000 K"/>',
           "quasar": "<QuasarSED/>"}[sed]
    path = str(tmp_path / (sed + ".ski"))
    with open(path, "w") as f:
        f.write(SKI % {"N": N, "SED": xml})
    r = O.run(path, rng=O.RNG_MT, threads=1, packages=100)
    got = r.seds[0][0]  # raw SED accumulator of the one SEDInstrument slot: L_ell
    lam, lo, hi = loggrid(0.005e-6, 2000e-6, N)
    ref = blackbody(float(sed[2:]), lo, hi) if sed.startswith("bb") else quasar(lam, lo, hi)
    ref = ref / ref.sum()
    np.testing.assert_allclose(got / got.sum(), ref, rtol=1e-12, atol=1e-300)
