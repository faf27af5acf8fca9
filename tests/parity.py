"""Element-wise parity of two tally tables (engine vs oracle on the same Philox streams) with an explicit
outlier budget.

Device libm (ocml) and glibc can differ in the last ulp of exp/log/cbrt/sincospi; very rarely that flips a
discrete decision (a cell boundary, a rejection test) and changes one packet's history. Such a packet moves
its luminosity between a few cells, so a same-stream comparison is judged by

* the outliers: elements whose relative difference exceeds rtol (their number and the largest relative
  difference among them are reported, and the number is held to an explicit budget);
* the outliers' mass: the summed |a - b| over them, relative to the table's total, held to `mass`.

Elements below `floor` x the table's maximum are not compared: in optically thick models the deepest cells
receive ~1e-220 of a packet's luminosity, where the engine's running exp(-tau) and the oracle's exp(-tau)
per segment underflow at different depths. Each report is appended to $SKIRT_PARITY_LOG (JSON lines) when
that variable is set, so a GPU run leaves the measured outlier counts behind.
"""
import json
import os

import numpy as np

# Outlier budgets of the same-stream tests: elements per table allowed beyond rtol (stellar phases at 1e-9,
# dust phases at 1e-8). Measured on MI355X (profiles/r02_parity_outliers.jsonl): no outlier in any table of
# any model, except the stellar Labs of the optically thick octree self-absorption models (pan_oct_sa,
# pan_oct_sac): 99 of 39082 cells, largest relative difference 4.5e-4, together 1.4e-19 of the total --
# cells at the bottom of the dynamic range, where the engine's running product of exp(-dtau) and the
# oracle's exp(-tau) per segment part in the last digits.
STELLAR_OUTLIERS = 0
DUST_OUTLIERS = 0
THICK_OUTLIERS = 128


def outliers(a, b, rtol, floor=1e-15):
    """(number of outliers, largest relative difference over the compared elements, outlier mass relative to
    the table's total, number of compared elements)."""
    a, b = np.asarray(a, dtype=np.float64).ravel(), np.asarray(b, dtype=np.float64).ravel()
    scale = np.maximum(np.abs(a), np.abs(b))
    top = scale.max() if scale.size else 0.0
    cmp = scale > floor * top
    diff = np.abs(a - b)
    rel = np.where(cmp, diff / np.where(scale > 0, scale, 1.0), 0.0)
    out = cmp & (rel > rtol)
    total = np.abs(b).sum()
    mass = diff[out].sum() / total if total > 0 else 0.0
    return int(out.sum()), float(rel.max() if rel.size else 0.0), float(mass), int(cmp.sum())


def assert_parity(a, b, rtol, budget, label, mass=1e-12, floor=1e-15):
    """Asserts at most `budget` outliers at rtol whose summed difference is at most `mass` of the total."""
    n, worst, m, ncmp = outliers(a, b, rtol, floor)
    test = os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0]
    rec = {"test": test, "label": label, "rtol": rtol, "outliers": n, "compared": ncmp, "max_rel": worst, "outlier_mass": m,
           "budget": budget}
    path = os.environ.get("SKIRT_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")
    print("parity %s: %d/%d outliers at rtol %g (max rel %.3g, mass %.3g)" % (label, n, ncmp, rtol, worst, m))
    assert n <= budget and m <= mass, rec
