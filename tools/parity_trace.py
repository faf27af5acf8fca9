"""Packet trace of a same-stream parity difference (tool only).

The 128^3 Cartesian model of tests/test_gpu_cartesian.py (pan_cart16 with 128 bins per axis, 257
wavelengths, 20 packages per wavelength) showed cells whose Labs differ from the oracle's by up to 1.3e-7
relative (profiles/r05_labs_over_4gib.txt). A cell's stellar Labs at wavelength ell receives adds only from
the packets of that wavelength, global indices ell * 20 ... ell * 20 + 19, so each packet is run alone:

  engine (GPU box):  SKIRT_AMD_LIB=libskirt_amd_dbgfill.so python tools/parity_trace.py engine OUT
                     (tools/build_variant.sh dbgfill -DSKIRT_DEBUG_FILL: the trace kernel prints every FILL
                     ray's start and its dust segments)
  oracle (here):     python tools/parity_trace.py oracle OUT   (ORACLE_DEBUG_FILL=1, one thread)
  compare (here):    python tools/parity_trace.py compare OUT

Each side writes OUT/<side>_<ell>_<p>.txt (the packet's FILL paths) and OUT/<side>_cells.json (the target
cells' Labs per packet). `compare` names the packet whose add differs and the first value in its history
that differs, with its ulp distance.
"""
import ctypes
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
GOLD = os.path.join(ROOT, "tests", "golden", "ski")
PACKAGES = 20
TARGETS = [(317912, 44), (449794, 73)]  # (reference cell, wavelength) of profiles/r05_labs_over_4gib.txt


def model_path():
    text = open(os.path.join(GOLD, "pan_cart16.ski")).read()
    for n in ("X", "Y", "Z"):
        text = text.replace('<mesh%s type="MoveableMesh"><LinMesh numBins="16"/></mesh%s>' % (n, n),
                            '<mesh%s type="MoveableMesh"><LinMesh numBins="128"/></mesh%s>' % (n, n))
    text = text.replace('points="10"', 'points="257"')
    path = "/tmp/parity_trace_cart128.ski"
    with open(path, "w") as f:
        f.write(text)
    return path


def capture(fn, out):
    """runs fn() with the process's fd 1 redirected into file `out` (device printf and C printf included)"""
    libc = ctypes.CDLL(None)
    libc.fflush(None)
    sys.stdout.flush()
    saved = os.dup(1)
    fd = os.open(out, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    os.dup2(fd, 1)
    os.close(fd)
    try:
        return fn()
    finally:
        libc.fflush(None)
        os.dup2(saved, 1)
        os.close(saved)


def run_engine(outdir):
    import numpy as np
    import skirt_amd as S

    sim = S.Simulation(model_path(), packages=PACKAGES)
    sim.attach(0)
    res = {}
    for cell, ell in TARGETS:
        for p in range(PACKAGES):
            g = ell * PACKAGES + p
            sim.zero_tallies()

            def one():
                sim.run_stellar(g, 1)
                sim.fetch()
            capture(one, os.path.join(outdir, "engine_%d_%d.txt" % (ell, p)))
            col = np.ascontiguousarray(sim.labs()[:, ell])
            res["%d_%d" % (ell, p)] = {"target": float(col[cell]), "nonzero": int(np.count_nonzero(col)),
                                       "sum": float(col.sum())}
            print("engine ell", ell, "packet", p, res["%d_%d" % (ell, p)], flush=True)
    with open(os.path.join(outdir, "engine_cells.json"), "w") as f:
        json.dump(res, f, indent=1)


def run_oracle(outdir):
    import numpy as np
    os.environ["ORACLE_DEBUG_FILL"] = "1"
    import oracle_lib as O

    path = model_path()
    res = {}
    for cell, ell in TARGETS:
        for p in range(PACKAGES):
            g = ell * PACKAGES + p
            box = {}

            def one():
                box["r"] = O.run(path, rng=O.RNG_PHILOX, threads=1, packages=PACKAGES, packet_begin=g,
                                 packet_end=g + 1, phases=O.PHASES_STELLAR)
            capture(one, os.path.join(outdir, "oracle_%d_%d.txt" % (ell, p)))
            col = np.ascontiguousarray(box["r"].labs[:, ell])
            res["%d_%d" % (ell, p)] = {"target": float(col[cell]), "nonzero": int(np.count_nonzero(col)),
                                       "sum": float(col.sum())}
            del box
            print("oracle ell", ell, "packet", p, res["%d_%d" % (ell, p)], flush=True)
    with open(os.path.join(outdir, "oracle_cells.json"), "w") as f:
        json.dump(res, f, indent=1)


def ulps(a, b):
    """distance of two doubles in units in the last place (same sign assumed)"""
    ia = struct.unpack("<q", struct.pack("<d", a))[0]
    ib = struct.unpack("<q", struct.pack("<d", b))[0]
    return abs(ia - ib)


def parse(fname):
    paths = []
    for line in open(fname):
        w = line.split()
        if len(w) < 2 or w[0] not in ("E", "O"):
            continue
        if w[1] == "L":
            paths.append({"ell": int(w[2]), "r": [float(v) for v in w[3:6]], "k": [float(v) for v in w[6:9]],
                          "L": float(w[9]), "segs": []})
        elif w[1] == "S":
            paths[-1]["segs"].append((int(w[2]), float(w[3]), float(w[4]), float(w[5])))
    return paths


def engine_cell_to_ref(m, n=128):
    """the engine's bricked Cartesian device number (Grid<SKIRT_GRID_CARTESIAN>::dev) -> k + n j + n^2 i"""
    b, o = m >> 3, m & 7
    bz = by = (n + 1) >> 1
    i2, rest = divmod(b, by * bz)
    j2, k2 = divmod(rest, bz)
    i, j, k = 2 * i2 + ((o >> 2) & 1), 2 * j2 + ((o >> 1) & 1), 2 * k2 + (o & 1)
    return k + n * j + n * n * i


def compare(outdir):
    eng = json.load(open(os.path.join(outdir, "engine_cells.json")))
    orc = json.load(open(os.path.join(outdir, "oracle_cells.json")))
    for cell, ell in TARGETS:
        print("== cell %d, wavelength %d" % (cell, ell))
        for p in range(PACKAGES):
            key = "%d_%d" % (ell, p)
            a, b = eng[key]["target"], orc[key]["target"]
            if a == 0 and b == 0:
                continue
            rel = abs(a - b) / max(abs(a), abs(b))
            print("  packet %d (global %d): engine %.17g oracle %.17g rel %.3g" % (p, ell * PACKAGES + p, a, b, rel))
            if rel < 1e-9:
                continue
            pe = parse(os.path.join(outdir, "engine_%d_%d.txt" % (ell, p)))
            po = parse(os.path.join(outdir, "oracle_%d_%d.txt" % (ell, p)))
            print("    FILL paths: engine %d, oracle %d" % (len(pe), len(po)))
            for n, (x, y) in enumerate(zip(pe, po)):
                du = [ulps(u, v) for u, v in zip(x["r"] + x["k"] + [x["L"]], y["r"] + y["k"] + [y["L"]])]
                se = [(engine_cell_to_ref(m), ds, dt, ad) for m, ds, dt, ad in x["segs"]]
                so = y["segs"]
                hit = [q for q, s in enumerate(se) if s[0] == cell] + [q for q, s in enumerate(so) if s[0] == cell]
                print("    path %d: start/direction/L ulps %s; segments engine %d oracle %d%s" %
                      (n, du, len(se), len(so), "; crosses the cell" if hit else ""))
                first = None
                for q in range(min(len(se), len(so))):
                    if se[q][0] != so[q][0]:
                        first = q
                        break
                if first is not None or len(se) != len(so):
                    q = first if first is not None else min(len(se), len(so))
                    print("      cell sequences part at segment %d:" % q)
                    for t in range(max(0, q - 2), min(max(len(se), len(so)), q + 3)):
                        e = se[t] if t < len(se) else None
                        o = so[t] if t < len(so) else None
                        print("        %d engine %s | oracle %s" % (t, e, o))
                for t in sorted(set(q for q, s in enumerate(se) if s[0] == cell) |
                                set(q for q, s in enumerate(so) if s[0] == cell)):
                    e = se[t] if t < len(se) else None
                    o = so[t] if t < len(so) else None
                    extra = ""
                    if e and o and e[0] == o[0]:
                        extra = " ds ulps %d rel %.3g; add rel %.3g" % (
                            ulps(e[1], o[1]), abs(e[1] - o[1]) / max(e[1], o[1]),
                            abs(e[3] - o[3]) / max(abs(e[3]), abs(o[3]), 1e-300))
                    print("      at the cell, segment %d: engine %s | oracle %s%s" % (t, e, o, extra))


if __name__ == "__main__":
    side, outdir = sys.argv[1], sys.argv[2]
    os.makedirs(outdir, exist_ok=True)
    {"engine": run_engine, "oracle": run_oracle, "compare": compare}[side](outdir)
