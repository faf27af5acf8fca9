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


def cartesian_neighbour_scale(table, shape):
    """For a Labs table (cells x wavelengths) of a Cartesian grid of shape (Nx, Ny, Nz), cell m = k + Nz j +
    Nz Ny i (CartesianDustGrid.cpp:305-308): a function (cells, ells) -> the largest |value| of each element's
    six face neighbours at the same wavelength (see `slivers` in assert_parity)."""
    nx, ny, nz = shape
    t = np.asarray(table)

    def scale(cells, ells):
        i, rem = np.divmod(cells, ny * nz)
        j, k = np.divmod(rem, nz)
        best = np.zeros(cells.size)
        for di, dj, dk in ((1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)):
            ii, jj, kk = i + di, j + dj, k + dk
            ok = (ii >= 0) & (ii < nx) & (jj >= 0) & (jj < ny) & (kk >= 0) & (kk < nz)
            m = np.where(ok, kk + nz * jj + nz * ny * ii, 0)
            best = np.maximum(best, np.where(ok, np.abs(t[m, ells]), 0.0))
        return best
    return scale


def assert_parity(a, b, rtol, budget, label, mass=1e-12, floor=1e-15, drift=100.0, drift_budget=None,
                  slivers=None):
    """Asserts at most `budget` outliers beyond drift x rtol, at most `drift_budget` (default 0.1 % of the
    compared elements) between rtol and drift x rtol (last-digit drift of long chains of segments), and
    that all of them together carry at most `mass` of the table's total.

    slivers (a function (cells, ells) -> scale, e.g. cartesian_neighbour_scale): an element beyond rtol whose
    difference is within rtol of that scale is a sliver, counted apart (at most 0.01 % of the compared
    elements) instead of as an outlier. A ray that passes a cell's edge within a hair's breadth crosses it
    over a sliver whose length is the difference of two nearly equal coordinates; the last-ulp differences
    of the position (the engine's exit distances are (x_E - x) * (1/k), the reference's (x_E - x) / k, and
    its launch directions come from other, equivalent formulas) then change the
    sliver's length, and a cell that only that sliver reaches, by up to ulp(x) / length relative. The same
    segment is a full crossing of the neighbouring cells, so its error is bounded relative to them
    (profiles/r06_parity_trace.txt traces such a cell on the 128^3 Cartesian model)."""
    if slivers is not None:
        a2, b2 = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
        scale = np.maximum(np.abs(a2), np.abs(b2))
        top = scale.max() if scale.size else 0.0
        diff = np.abs(a2 - b2)
        cand = np.argwhere((scale > floor * top) & (diff > rtol * scale))
        nsl = 0
        if cand.size:
            nb = slivers(cand[:, 0], cand[:, 1])
            sl = diff[cand[:, 0], cand[:, 1]] <= rtol * nb
            nsl = int(sl.sum())
            # the slivers compared as equal: the oracle's value in place of the engine's
            a2 = a2.copy()
            a2[cand[sl, 0], cand[sl, 1]] = b2[cand[sl, 0], cand[sl, 1]]
            print("parity %s: %d sliver element(s), difference within %g of their neighbours" % (label, nsl, rtol))
        assert nsl <= max(1, (scale > floor * top).sum() // 10000), nsl
        a = a2
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
