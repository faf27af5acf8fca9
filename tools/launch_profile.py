"""Per-launch view of a rocprofv3 kernel trace of bench.py (one step): the photon kernels' launches in time
order, the GPU's idle time between them (host round trips, launch latency), and the trace launches by
duration (how much of the step the short tail launches of each phase take).
Usage: python tools/launch_profile.py <rocprofv3 output dir> <steps in the run>"""
import csv
import glob
import sys


def main():
    rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0])))
    steps = int(sys.argv[2])
    ks = []
    for r in rows:
        n = r["Kernel_Name"]
        for k in ("traceKernel", "eventKernel", "detectKernel", "contKernel"):
            if k in n:
                ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
                break
        else:
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "other"))
    ks.sort()
    ntrace = sum(1 for k in ks if k[2] == "traceKernel")
    per = ntrace // (steps + 1)  # warmup step + timed steps
    # the last step: its trace launches are the last `per`
    tr = [i for i, k in enumerate(ks) if k[2] == "traceKernel"]
    first = tr[-per]
    # include the event kernel right before the step's first trace launch
    while first > 0 and ks[first - 1][2] in ("eventKernel", "detectKernel", "other"):
        first -= 1
        if ks[first][2] == "eventKernel":
            break
    ph = ks[first:]
    t0, t1 = ph[0][0], max(e for _, e, _ in ph)
    ev = sorted([(s, 1) for s, _, _ in ph] + [(e, -1) for _, e, _ in ph])
    depth, last, union = 0, t0, 0
    for t, d in ev:
        if depth > 0:
            union += t - last
        depth += d
        last = t
    busy = {}
    for s, e, k in ph:
        busy[k] = busy.get(k, 0) + (e - s)
    print("last step: %.1f ms wall, GPU busy %.1f ms, idle %.1f ms (%.1f %%), %d trace launches" % (
        (t1 - t0) / 1e6, union / 1e6, (t1 - t0 - union) / 1e6, 100 * (t1 - t0 - union) / (t1 - t0), per))
    for k, v in sorted(busy.items(), key=lambda x: -x[1]):
        print("  %-12s %8.1f ms" % (k, v / 1e6))
    durs = sorted(((e - s) / 1e6 for s, e, k in ph if k == "traceKernel"), reverse=True)
    edges = [1e9, 20, 5, 1, 0.2, 0.05, 0]
    for hi, lo in zip(edges, edges[1:]):
        sel = [d for d in durs if lo <= d < hi]
        if sel:
            print("  trace launches in [%g, %g) ms: %3d, %8.1f ms" % (lo, hi, len(sel), sum(sel)))
    # sequence, compact
    seq = []
    for s, e, k in ph:
        if k == "traceKernel":
            seq.append("%.2f" % ((e - s) / 1e6))
    print("trace launch durations (ms, in order):", " ".join(seq))


if __name__ == "__main__":
    main()
