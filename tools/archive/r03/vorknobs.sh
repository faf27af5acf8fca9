# round 3: Voronoi trace kernel knobs at the new bounds: entries per load round (4, 8, 12, 16), 3 waves/SIMD
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/vorknobs.txt
: > $out
for v in new u4 u12 u16 w3 new; do
  lib=libskirt_amd.so; [ $v != new ] && lib=libskirt_amd_$v.so
  SKIRT_AMD_LIB=$lib timeout -k 10 200 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/vk_$v.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/vk_$v.log; exit 1; }
  python - "c4 $v" gpurun_out/vk_$v.log >> $out <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("%-10s %.4e pkt/s  %.1f ms/step  trace %.3f ms x %d" % (sys.argv[1], r["value"], r["ms_per_step"], r["roofline"]["launch_ms_avg"], r["roofline"]["launches_per_step"]))
PY
  tail -1 $out
done
