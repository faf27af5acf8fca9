"""Summarise a tools/gpu_prof.sh run (rocprofv3 CSVs under gpurun_out/prof_<cfg>/) into profiles/:

  profiles/<round>_rocprof_<cfg>_kernel_stats.csv   the --kernel-trace --stats summary, as written
  profiles/<round>_rocprof_<cfg>.txt                per-kernel averages of every PMC counter collected
  profiles/pmc_<cfg>.json                           per traceKernel launch: HBM bytes, VALU/SALU wave-instructions,
                                                    f64 atomic requests, GRBM_GUI_ACTIVE (read by bench.py)

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE come from separate passes
(they cannot share one on gfx950), in KiB; WRITE_SIZE is exact for 16-byte stores and for the f64
atomics. The guide's halving of FETCH_SIZE holds for coalesced 16-byte-per-lane streams only; a
scattered gather (one lane per 64-byte line, the trace kernel's leaf-map, Labs and neighbour loads)
reports its whole 64-byte line (tools/gather_bench.hip, profiles/r02_gather_calibration.txt), so
FETCH_SIZE is taken as it is: traffic = FETCH_SIZE + WRITE_SIZE.
usage: python tools/pmc_traffic.py <cfg> <round> [<tag>]
  a tag (a variant's gpurun_out/prof_<cfg><tag>, e.g. tools/gpu_prof.sh run with TAG=_cache1) writes
  profiles/<round>_rocprof_<cfg><tag>.* and leaves pmc_<cfg>.json (the bench's default build) alone
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(pattern):
    hits = glob.glob(pattern, recursive=True)
    return hits[0] if hits else None


def counters(path):
    """{kernel: {counter: [per-dispatch values]}}"""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        key = (r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    for (d, cn), v in per.items():
        out[names[d]][cn].append(v)
    return out


def short(name):
    for k in ("traceKernel", "eventKernel", "detectKernel", "buildLeafMapKernel"):
        if k in name:
            return k
    return name[:40]


def main():
    cfg, rnd = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else ""
    base = os.path.join(REPO, "gpurun_out", "prof_" + cfg + tag)
    prof = os.path.join(REPO, "profiles")
    stats = one(base + "/trace/**/*kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, "%s_rocprof_%s%s_kernel_stats.csv" % (rnd, cfg, tag)))
    lines = ["rocprofv3 summary, config %s (%s)" % (cfg, open(os.path.join(base, "cmd.txt")).read().strip()
                                                   if os.path.exists(os.path.join(base, "cmd.txt")) else ""), ""]
    lines.append("kernel stats (--kernel-trace --stats):")
    for r in csv.DictReader(open(stats)):
        lines.append("  %-20s calls %6s  avg %9.3f us  total %9.3f ms  %5.1f %%" % (
            short(r["Name"]), r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6,
            float(r["Percentage"])))
    avg = {}
    for d in sorted(glob.glob(base + "/*/")):
        path = one(d + "**/*counter_collection.csv")
        if not path:
            continue
        lines.append("")
        lines.append("PMC pass %s (per-dispatch averages):" % os.path.basename(d.rstrip("/")))
        # every dispatch of a kernel family (traceKernel<...>, traceKernelNoStore<...>, traceKernelVor<...>:
        # one average per trace launch, as bench.py times them) pooled
        pooled = collections.defaultdict(lambda: collections.defaultdict(list))
        for k, cs in counters(path).items():
            for cn, vals in cs.items():
                pooled[short(k)][cn].extend(vals)
        for k, cs in sorted(pooled.items()):
            for cn, vals in sorted(cs.items()):
                m = sum(vals) / len(vals)
                avg[(k, cn)] = m
                lines.append("  %-20s %-22s %.6g  (%d dispatches)" % (k, cn, m, len(vals)))
    open(os.path.join(prof, "%s_rocprof_%s%s.txt" % (rnd, cfg, tag)), "w").write("\n".join(lines) + "\n")
    f = avg.get(("traceKernel", "FETCH_SIZE"))
    w = avg.get(("traceKernel", "WRITE_SIZE"))
    if f is not None and w is not None and not tag:
        d = {"kernel": "traceKernel", "fetch_size_kib": f, "write_size_kib": w,
             "traffic_bytes_per_launch": f * 1024 + w * 1024,
             "source": "profiles/%s_rocprof_%s.txt: FETCH_SIZE + WRITE_SIZE per traceKernel dispatch" % (rnd, cfg)}
        # the issue and atomic counters of the same dispatches, where their passes ran
        for key, cn in (("valu_insts_per_launch", "SQ_INSTS_VALU"), ("salu_insts_per_launch", "SQ_INSTS_SALU"),
                        ("atomic_requests_per_launch", "TCC_EA0_ATOMIC_sum"), ("grbm_gui_active_per_launch", "GRBM_GUI_ACTIVE"),
                        ("sq_waves_per_launch", "SQ_WAVES"), ("valu_active_quads_per_launch", "SQ_ACTIVE_INST_VALU"),
                        ("inst_active_quads_per_launch", "SQ_ACTIVE_INST_ANY"), ("wave_quads_per_launch", "SQ_WAVE_CYCLES")):
            v = avg.get(("traceKernel", cn))
            if v is not None:
                d[key] = v
        json.dump(d, open(os.path.join(prof, "pmc_%s.json" % cfg), "w"), indent=1)
        print(json.dumps(d))
    print("\n".join(lines))


if __name__ == "__main__":
    main()
