"""Overlap analysis of a rocprofv3 kernel trace (a kernel trace, e.g. rocprofv3 --kernel-trace): per kernel busy time, the
union of busy intervals, and how much of the last timed phase two kernels overlapped."""
import csv
import glob
import sys

rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0])))
ks = []
for r in rows:
    n = r["Kernel_Name"]
    for k in ("traceKernel", "eventKernel", "detectKernel"):
        if k in n:
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
ks.sort()
# the last phase: kernels after the last gap > 5 ms
start = 0
for i in range(1, len(ks)):
    if ks[i][0] - max(e for _, e, _ in ks[:i]) > 5e6:
        start = i
ph = ks[start:]
t0, t1 = ph[0][0], max(e for _, e, _ in ph)
busy = {}
for s, e, k in ph:
    busy[k] = busy.get(k, 0) + (e - s)
ev = sorted([(s, 1) for s, _, _ in ph] + [(e, -1) for _, e, _ in ph])
depth, last, union, multi = 0, t0, 0, 0
for t, d in ev:
    if depth > 0:
        union += t - last
    if depth > 1:
        multi += t - last
    depth += d
    last = t
print("phase %.2f ms, kernels %d, union busy %.2f ms, >1 kernel running %.2f ms" % ((t1 - t0) / 1e6, len(ph), union / 1e6, multi / 1e6))
for k, v in sorted(busy.items()):
    print("  %-14s %.2f ms summed" % (k, v / 1e6))
for s, e, k in ph[:12]:
    print("  %8.3f %8.3f %s" % ((s - t0) / 1e6, (e - t0) / 1e6, k))
