"""Element-wise parity of two tally tables (engine vs oracle on the same Philox streams) with an explicit
outlier budget.

Device libm (ocml) and glibc can differ in the last ulp of exp/log/cbrt/sincospi; very rarely that flips a
discrete decision (a cell boundary, a rejection test) and changes one packet's history. Such a packet moves
its luminosity between a few cells, so a same-stream comparison is judged by

* the outliers: elements whose relative difference exceeds 100 x rtol (their number and the largest
  relative difference are reported, and the number is held to an explicit budget);
* the drift: elements between rtol and 100 x rtol, the last digits of long chains of segments parting
  (reported; at most 0.1 % of the table);
* the mass of both: the summed |a - b| over them, relative to the table's total, held to `mass`.

Elements below `floor` x the table's maximum are not compared: in optically thick models the deepest cells
receive ~1e-220 of a packet's luminosity, where device and host exp underflow at slightly different depths. Each report is appended to $SKIRT_PARITY_LOG (JSON lines) when
that variable is set, so a GPU run leaves the measured outlier counts behind.
"""
import json
import os

import numpy as np

# Outlier budgets of the same-stream tests: elements per table allowed beyond 100 x rtol (stellar phases
# at rtol 1e-9, dust phases at 1e-8). Measured on MI355X (profiles/r02_parity_outliers.jsonl,
# profiles/r03_gpu_tests_full.log): no element beyond rtol in any table of any fixture model; on the full C3
# octree 2 of 67,011 cells at 1.1e-9 (drift). Until round 3 the stellar Labs of the optically thick (3e6
# Msun) octree self-absorption models (pan_oct_sa, pan_oct_sac) differed in 32 of 39,082 cells beyond 1e-7
# (largest 4.5e-4, together 1.4e-19 of the total), with a budget of 128. Named cause: the engine carried a
# path's exp(-tau_{n-1}) as the running product of 1 - (-expm1(-dtau)) where the reference evaluates
# exp(-taustart) per segment (MonteCarloSimulation.cpp:458-462); behind a segment of dtau = 30 the product
# keeps only 1e-16 / exp(-30) = 1.7e-4 relative accuracy (tests/test_attenuation.py shows it on the CPU).
# The engine now evaluates exp(-taustart) per segment as the reference does, and those models have no
# element beyond 1e-9 either: one budget for all.
STELLAR_OUTLIERS = 0
DUST_OUTLIERS = 0


def outliers(a, b, rtol, floor=1e-15, drift=100.0):
    """(number of outliers -- elements beyond drift x rtol --, number of elements between rtol and
    drift x rtol, largest relative difference over the compared elements, outlier mass relative to the
    table's total, number of compared elements)."""
    a, b = np.asarray(a, dtype=np.float64).ravel(), np.asarray(b, dtype=np.float64).ravel()
    scale = np.maximum(np.abs(a), np.abs(b))
    top = scale.max() if scale.size else 0.0
    cmp = scale > floor * top
    diff = np.abs(a - b)
    rel = np.where(cmp, diff / np.where(scale > 0, scale, 1.0), 0.0)
    out = cmp & (rel > drift * rtol)
    near = cmp & (rel > rtol) & ~out
    total = np.abs(b).sum()
    mass = diff[out | near].sum() / total if total > 0 else 0.0
    return int(out.sum()), int(near.sum()), float(rel.max() if rel.size else 0.0), float(mass), int(cmp.sum())


def assert_parity(a, b, rtol, budget, label, mass=1e-12, floor=1e-15, drift=100.0, drift_budget=None):
    """Asserts at most `budget` outliers beyond drift x rtol, at most `drift_budget` (default 0.1 % of the
    compared elements) between rtol and drift x rtol (last-digit drift of long chains of segments), and
    that all of them together carry at most `mass` of the table's total."""
    n, nnear, worst, m, ncmp = outliers(a, b, rtol, floor, drift)
    test = os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0]
    rec = {"test": test, "label": label, "rtol": rtol, "outliers": n, "drift": nnear, "compared": ncmp,
           "max_rel": worst, "outlier_mass": m, "budget": budget}
    path = os.environ.get("SKIRT_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")
    print("parity %s: %d/%d outliers beyond %g, %d beyond %g (max rel %.3g, mass %.3g)" % (
        label, n, ncmp, drift * rtol, nnear, rtol, worst, m))
    if drift_budget is None:
        drift_budget = max(1, ncmp // 1000)
    assert n <= budget and nnear <= drift_budget and m <= mass, rec
