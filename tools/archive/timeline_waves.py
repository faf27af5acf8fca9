"""Per-wave timeline of one photon phase (SKIRT_EXPERIMENT_TIMELINE build, SKIRT_AMD_TIMELINE_OUT file):
# (archived in round 5: the SKIRT_EXPERIMENT_TIMELINE instrumentation was removed from engine.hip; git history keeps it)
per iteration the event, trace and detect kernels' spans, the gaps between them, and the trace kernel's
drain tail (from the first wave that found the ray queue exhausted to the last wave's end), with the
share of trace waves still running at 25/50/75 % of the tail.

usage: python tools/timeline_waves.py FILE"""
import struct
import sys

import numpy as np

TICK_US = 0.01  # s_memrealtime: 100 MHz


def main(path):
    with open(path, "rb") as f:
        kinds, launches, waves, its = struct.unpack("4i", f.read(16))
        words = 4
        rest = f.read()
        if (len(rest) - 4) % (kinds * launches * waves * 8) == 0:  # header with the record size
            words = struct.unpack("i", rest[:4])[0]
            rest = rest[4:]
        d = np.frombuffer(rest, dtype=np.uint64).reshape(kinds, launches, waves, words).astype(np.int64)
    n = min(its, launches)
    t0 = None
    rows = []
    for k in range(n):
        spans = []
        for kind in range(3):
            w = d[kind, k]
            w = w[w[:, 2] > 0]
            spans.append(w)
        tr, ev, de = spans
        if len(tr) == 0:
            continue
        if t0 is None:
            t0 = ev[:, 0].min() if len(ev) else tr[:, 0].min()
        e0, e1 = (ev[:, 0].min(), ev[:, 2].max()) if len(ev) else (0, 0)
        s0, s1 = tr[:, 0].min(), tr[:, 2].max()
        ex = tr[:, 1][tr[:, 1] > 0]
        x0 = ex.min() if len(ex) else s1
        tail = s1 - x0
        frac = []
        for q in (0.25, 0.5, 0.75):
            t = x0 + q * tail
            frac.append(np.mean(tr[:, 2] > t))
        d0, d1 = (de[:, 0].min(), de[:, 2].max()) if len(de) else (s1, s1)
        rows.append((k, (e1 - e0) * TICK_US, (s0 - e1) * TICK_US, (s1 - s0) * TICK_US, tail * TICK_US, frac,
                     (d0 - s1) * TICK_US, (d1 - d0) * TICK_US, int(tr[:, 3].sum())))
    print("it  event_us  gap_us  trace_us  tail_us  running@25/50/75%   gap_us  detect_us  rays")
    for r in rows:
        print("%2d %9.1f %7.1f %9.1f %8.1f   %.2f/%.2f/%.2f   %7.1f %9.1f  %d" % (
            r[0], r[1], r[2], r[3], r[4], r[5][0], r[5][1], r[5][2], r[6], r[7], r[8]))
    if d.shape[3] >= 8:  # event kernel: shader cycles per part of a round, summed over waves and iterations
        ev = d[1, :n]
        parts = ev[..., 4:8].sum(axis=(0, 1)).astype(float)
        names = ("loads+FILL/WALK events", "claims+launches", "block reservations", "ray/state writes")
        tot = parts.sum()
        print("event kernel round parts: " + ", ".join("%s %.1f%%" % (nm, 100 * v / tot) for nm, v in zip(names, parts)))
        print("event kernel round parts, wave-cycles x1e9: " + ", ".join("%s %.2f" % (nm, v / 1e9) for nm, v in zip(names, parts)))
    a = np.array([(r[1], r[2], r[3], r[4], r[6], r[7]) for r in rows])
    print("sum: event %.1f ms, gaps %.1f ms, trace %.1f ms (tail %.1f ms), detect %.1f ms" % (
        a[:, 0].sum() / 1e3, (a[:, 1].sum() + a[:, 4].sum()) / 1e3, a[:, 2].sum() / 1e3, a[:, 3].sum() / 1e3,
        a[:, 5].sum() / 1e3))


if __name__ == "__main__":
    main(sys.argv[1])
