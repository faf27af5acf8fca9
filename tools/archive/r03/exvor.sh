# round 3: Voronoi entry groups with exp(-tau) per FILL segment: p6 (new, 28 B/lane spilled), p4, one group
# of 8 (exnp8), against the product form at p6 (sm); C4 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/exvor.txt
: > $out
for v in new exp4 exnp8 sm new exp4 exnp8 sm; do
  lib=libskirt_amd.so; [ $v != new ] && lib=libskirt_amd_$v.so
  SKIRT_AMD_LIB=$lib timeout -k 10 200 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/xv_$v.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/xv_$v.log; exit 1; }
  python - "c4 $v" gpurun_out/xv_$v.log >> $out <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("%-10s %.4e pkt/s  %.1f ms/step  trace %.3f ms x %d" % (sys.argv[1], r["value"], r["ms_per_step"], r["roofline"]["launch_ms_avg"], r["roofline"]["launches_per_step"]))
PY
  tail -1 $out
done
