"""The attenuation exp(-tau_{n-1}) of the absorption sum along a FILL path, and how the engine's form of it
parts from the reference's (tests/parity.py).

The reference sums a packet's absorption with exp(-taustart) per segment (MonteCarloSimulation.cpp:458-462).
Until round 3 the engine carried exp(-tau) as the running product of 1 - (-expm1(-dtau)) over the path. Both
agree to a few ulp per factor while dtau is small. Behind an optically thick segment, 1 - (1 - exp(-dtau))
cancels: the product keeps only about 1e-16 / exp(-dtau) relative accuracy (dtau = 30: 1.7e-4). These tests
reproduce that on the CPU, with the oracle switched to the product form (oracle_set_engine_attenuation mode 1):
a few tens of deep cells on the 3e6 Msun pan_oct_sa models, with a mass below 1e-18 of the table, as the GPU
showed then; the thin models show none.

Since round 5 the engine carries a hybrid (Tracer::segment, kCarryTau = 0.5): f <- f - f * (-expm1(-dtau))
while dtau < 0.5, where the product is exact to about an ulp per segment, and exp(-tau) evaluated anew after a
thicker segment, where the product would cancel. The oracle's mode 2 is that arithmetic;
test_hybrid_carry_keeps_the_thick_models_deep_cells shows it gives no such outliers, and the GPU's thick-model
Labs equal the oracle's (reference form) to 1e-9 with no outlier (test_dust_phases_match_oracle_same_streams)."""
import os

import numpy as np

import oracle_lib as O
from parity import outliers

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ski")


def test_product_of_complements_cancels_behind_thick_segments():
    rel = []
    for dtau in (1.0, 10.0, 20.0, 30.0):
        prod = 1.0 - (-np.expm1(-dtau))
        rel.append(abs(prod - np.exp(-dtau)) / np.exp(-dtau))
    assert rel[0] < 1e-15 and rel[1] < 1e-12
    assert 1e-9 < rel[2] < 1e-6 and rel[3] > 1e-5


def _labs(name, product):
    path = os.path.join(GOLD, name + ".ski")
    if product:
        with O.engine_attenuation():
            return O.run(path, rng=O.RNG_PHILOX, threads=8, packages=300).labs
    return O.run(path, rng=O.RNG_PHILOX, threads=8, packages=300).labs


def test_engine_attenuation_form_changes_only_deep_cells_of_thick_models():
    # thin octree model: the two forms agree to rounding
    n, _, worst, _, _ = outliers(_labs("pan_oct", False), _labs("pan_oct", True), 1e-9)
    assert n == 0 and worst < 1e-12
    # the thick (3e6 Msun) self-absorption model: outliers, all in cells of negligible mass
    n, drift, worst, mass, cmp = outliers(_labs("pan_oct_sa", False), _labs("pan_oct_sa", True), 1e-9)
    assert 0 < n + drift < 0.01 * cmp
    assert 1e-7 < worst < 1e-2
    assert mass < 1e-18


def test_hybrid_carry_keeps_the_thick_models_deep_cells():
    """the engine's carry since round 5 (oracle mode 2) against the reference's exp(-taustart): no element of
    the thick pan_oct_sa model's Labs beyond 1e-9 (the product form, mode 1, puts tens of deep cells there)"""
    path = os.path.join(GOLD, "pan_oct_sa.ski")
    ref = O.run(path, rng=O.RNG_PHILOX, threads=8, packages=300).labs
    with O.engine_attenuation(2):
        hybrid = O.run(path, rng=O.RNG_PHILOX, threads=8, packages=300).labs
    np.testing.assert_allclose(hybrid, ref, rtol=1e-9, atol=1e-300)
