# round 3: PMC counters of the C4 trace kernel, new vs base Voronoi step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/vorprof
for v in new base; do
  lib=libskirt_amd.so; [ $v = base ] && lib=libskirt_amd_base.so
  SKIRT_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/vorprof/$v -o run -- python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/vorprof/$v.log 2>&1 || { echo FAIL $v; tail -3 gpurun_out/vorprof/$v.log; exit 1; }
  python3 - gpurun_out/vorprof/$v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
per = collections.defaultdict(float); names = {}
for r in csv.DictReader(open(f)):
    if "traceKernelVor" not in r["Kernel_Name"]: continue
    per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
tot = collections.defaultdict(float); n = len({d for d, _ in per})
for (d, c), v in per.items(): tot[c] += v
print(sys.argv[1], "dispatches", n, " ".join("%s=%.4g" % (c, v / n) for c, v in sorted(tot.items())))
PY
done
