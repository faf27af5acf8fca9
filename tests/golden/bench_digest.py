"""Digests of the reference's outputs for the BASELINE benchmark models (test infrastructure).

The four benchmarks/*.ski models are run by the rebuilt reference (`skirt -t 1`, oracle/ref.mk) at 1e3
packages per wavelength with the diagnostic outputs on (make_bench_fixtures.sh). Their frames and per-cell
tables are large (a 250 x 250 x 25 float32 cube, 622,490 cell rows for C3), so tests/golden/ref/bench/
keeps the small files whole (SEDs, ds_convergence, ds_crossed, the log excerpt) and, per large file, a digest:

  FITS frames   shape, SHA-256 of the float32 data as written (big-endian), per-wavelength sums
  ds_cellprops  rows, SHA-256 of the rows' text tokens (and of each column's), per-column sums

Equal SHA-256 values mean bit-for-bit equal outputs, which is what the oracle in MT mode must produce
(tests/test_oracle_golden.py::test_oracle_matches_reference_on_the_benchmark_models).
usage: python bench_digest.py <output dir> <tag>   (prints the digest JSON)
"""
import glob
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import skirt_files as F  # noqa: E402

BIG = ("_total.fits", "_ds_cellprops.dat")


def fits_digest(path):
    raw = open(path, "rb").read()
    a = F.read_fits(path)
    n = a.size * 4
    # the data follow the header's 2880-byte blocks: the last n bytes before the padding
    off = raw.find(b"END" + b" " * 77)
    off = (off // 2880 + 1) * 2880
    data = raw[off:off + n]
    return {"shape": list(a.shape), "sha256": hashlib.sha256(data).hexdigest(),
            "sums": [float(x) for x in a.astype(np.float64).reshape(a.shape[0], -1).sum(axis=1)]}


def cellprops_digest(path):
    rows = [l.split() for l in open(path) if l.strip() and not l.startswith("#")]
    h = hashlib.sha256()
    for r in rows:
        h.update((" ".join(r) + "\n").encode())
    ncol = len(rows[0]) if rows else 0
    hc = [hashlib.sha256() for _ in range(ncol)]
    for r in rows:
        for q in range(ncol):
            hc[q].update((r[q] + "\n").encode())
    cols = np.array([[float(x) for x in r] for r in rows]) if rows else np.zeros((0, 0))
    return {"rows": len(rows), "sha256": h.hexdigest(), "sha256_columns": [x.hexdigest() for x in hc],
            "sums": [float(x) for x in cols.sum(axis=0)]}


def digest(outdir, tag):
    out = {}
    for path in sorted(glob.glob(os.path.join(outdir, tag + "_*"))):
        base = os.path.basename(path)
        if base.endswith("_total.fits"):
            out[base] = fits_digest(path)
        elif base.endswith("_ds_cellprops.dat"):
            out[base] = cellprops_digest(path)
    return out


if __name__ == "__main__":
    print(json.dumps(digest(sys.argv[1], sys.argv[2]), indent=1, sort_keys=True))
