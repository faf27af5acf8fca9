#!/usr/bin/env python3
"""Convert the reference's tabulated resource data (dat/) into compact binary tables.

The reference reads these text tables at setup time (SKIRTcore/SunSED.cpp setupSelfBefore,
SKIRTcore/OligoStellarComp.cpp setupSelfBefore, SKIRTcore/InterstellarDustMix.cpp setupSelfBefore).
The GPU box has no /root/reference, so the numeric tables travel with the package as raw little-endian
float64 arrays. The numbers are the parsed text values themselves (strtod and Python float() are both
correctly rounded), in file order and before any unit conversion; the C++ loader applies the same
conversions as the reference code.

Layout of every .bin file: int64 nrows, int64 ncols, then nrows*ncols float64 (row-major).

Usage: python tools/convert_dat.py [/root/reference/dat] [skirt_amd/data]
"""
import os
import struct
import sys


def read_rows(path, skip_header_lines=0, comment="#"):
    rows = []
    with open(path) as f:
        lines = f.read().splitlines()
    for i, line in enumerate(lines):
        if i < skip_header_lines:
            continue
        s = line.strip()
        if not s or s.startswith(comment):
            continue
        rows.append([float(t) for t in s.split()])
    return rows


def write_bin(path, rows):
    ncols = len(rows[0])
    assert all(len(r) == ncols for r in rows)
    with open(path, "wb") as f:
        f.write(struct.pack("<qq", len(rows), ncols))
        for r in rows:
            f.write(struct.pack("<%dd" % ncols, *r))


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/dat"
    dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(__file__), "..", "skirt_amd", "data")
    os.makedirs(dst, exist_ok=True)

    # SunSED.dat: one header line, then the count, then (lambda [micron], L [W/micron]) pairs
    rows = read_rows(os.path.join(src, "SED/Sun/SunSED.dat"))
    count = int(rows[0][0])
    pairs = rows[1:]
    assert len(pairs) == count, (len(pairs), count)
    write_bin(os.path.join(dst, "SunSED.bin"), pairs)

    # InterstellarDustMix.dat: '#' header lines, then 1064 rows of
    # lambda [micron], albedo, <cos>, C_ext/H, K_abs [cm2/g], <cos^2> (longest wavelength first)
    rows = read_rows(os.path.join(src, "DustMix/InterstellarDustMix.dat"))
    assert len(rows) == 1064, len(rows)
    write_bin(os.path.join(dst, "InterstellarDustMix.bin"), rows)

    # MeanZubkoDustMix.dat: '#' header lines, then rows of lambda [micron], Cabs, Csca, tau [cm2/H], albedo,
    # g; MeanZubkoDustMix.cpp reads the first 1201 of them
    rows = read_rows(os.path.join(src, "DustMix/MeanZubkoDustMix.dat"))
    assert len(rows) >= 1201, len(rows)
    write_bin(os.path.join(dst, "MeanZubkoDustMix.bin"), rows[:1201])

    # DraineLiDustMix.dat: '#' header lines, then 800 rows of lambda [micron], Cabs, Csca [cm2/H], emission,
    # albedo, g (DraineLiDustMix.cpp)
    rows = read_rows(os.path.join(src, "DustMix/DraineLiDustMix.dat"))
    assert len(rows) >= 800, len(rows)
    write_bin(os.path.join(dst, "DraineLiDustMix.bin"), rows[:800])
    print("wrote", dst)


if __name__ == "__main__":
    main()
