"""continuousScattering (MonteCarloSimulation::continuouspeeloffscattering, MonteCarloSimulation.cpp:367-434)
in the oracle: peel-offs from a random point of every dust segment of each path replace the peel-off at
the interaction point. The reference fixtures pan_cart16_cs, pan_oct_cs and vor_pan_cs pin it (tests/test_oracle_golden.py); both
estimators measure the same scattered flux, so the oracle's continuous runs must agree with its own
discrete runs -- which are pinned bit for bit to the reference -- where the discrete estimator is well
sampled, while the continuous one also reaches the optically thin wavelengths where discrete packets
fall below the weight threshold before they scatter."""
import os

import numpy as np

import oracle_lib as O

SKI = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ski")


def _seds(name, seeds):
    return np.array([O.run(os.path.join(SKI, name + ".ski"), rng=O.RNG_PHILOX, threads=8, packages=2000, seed=sd,
                           phases=O.PHASES_ALL).seds[0] for sd in seeds])


def test_continuous_and_discrete_scattering_estimate_the_same_flux():
    seeds = [500 + k for k in range(12)]
    cont, disc = _seds("pan_cart16_cs", seeds), _seds("pan_cart16", seeds)
    np.testing.assert_array_equal(cont[:, 0], disc[:, 0])  # transparent flux: no dust, no draws
    for slot in (2, 4, 5):  # scattered stellar, scattered dust, first scattering level
        mc, sc = cont[:, slot].mean(0), cont[:, slot].std(0, ddof=1) / np.sqrt(len(seeds))
        md, sd = disc[:, slot].mean(0), disc[:, slot].std(0, ddof=1) / np.sqrt(len(seeds))
        good = (md > 0) & (sd < 0.2 * md)
        assert good.sum() >= 2
        z = (mc[good] - md[good]) / np.sqrt(sc[good] ** 2 + sd[good] ** 2)
        assert np.all(np.abs(z) < 4.5), (slot, z)
    # the thin wavelengths: scattered light only with the continuous peel-off
    thin = (disc[:, 2].max(axis=0) == 0)
    assert thin.any() and np.all(cont[:, 2].mean(axis=0)[thin][:2] > 0)
