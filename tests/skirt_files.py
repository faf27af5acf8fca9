"""Readers for SKIRT-format output files (SED text, FITS frames, ds_isrf, ds_cellprops)."""
import numpy as np


def read_text_table(path):
    rows = []
    with open(path) as f:
        for line in f:
            s = line.strip()
            if s and not s.startswith("#"):
                rows.append([float(t) for t in s.split()])
    return np.array(rows, dtype=np.float64)


def read_text_tokens(path):
    """Data rows as lists of the exact printed tokens (for digit-for-digit comparisons)."""
    rows = []
    with open(path) as f:
        for line in f:
            s = line.strip()
            if s and not s.startswith("#"):
                rows.append(s.split())
    return rows


def read_fits(path):
    """Primary-HDU image of a BITPIX=-32 FITS file as a float32 array shaped (NAXIS3, NAXIS2, NAXIS1)."""
    with open(path, "rb") as f:
        raw = f.read()
    hdr = {}
    off = 0
    while True:
        block = raw[off:off + 2880]
        off += 2880
        done = False
        for i in range(36):
            card = block[80 * i:80 * (i + 1)].decode("ascii")
            key = card[:8].strip()
            if key == "END":
                done = True
                break
            if card[8:10] == "= ":
                val = card[10:].split("/")[0].strip()
                hdr[key] = val
        if done:
            break
    assert int(hdr["BITPIX"]) == -32, hdr["BITPIX"]
    naxis = int(hdr["NAXIS"])
    dims = [int(hdr["NAXIS%d" % (i + 1)]) for i in range(naxis)]
    n = int(np.prod(dims))
    data = np.frombuffer(raw[off:off + 4 * n], dtype=">f4").astype(np.float32)
    return data.reshape(list(reversed(dims)) if naxis > 2 else [1] + list(reversed(dims)))
