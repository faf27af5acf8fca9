# round 3: the neighbour-parallel Voronoi drain step -- Voronoi parity (same streams, counts) and C4 A/B
# against the lane-serial step (wide0) and narrower thresholds (wide4, wide8)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_counts.py -k "vor" > gpurun_out/wide_tests.log 2>&1 || { tail -40 gpurun_out/wide_tests.log; exit 1; }
tail -3 gpurun_out/wide_tests.log
out=gpurun_out/wide.txt
: > $out
for v in new wide0 wide4 wide8 new wide0; do
  lib=libskirt_amd.so; [ $v != new ] && lib=libskirt_amd_$v.so
  SKIRT_AMD_LIB=$lib timeout -k 10 200 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wd_$v.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/wd_$v.log; exit 1; }
  python - "c4 $v" gpurun_out/wd_$v.log >> $out <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("%-10s %.4e pkt/s  %.1f ms/step  trace %.3f ms x %d" % (sys.argv[1], r["value"], r["ms_per_step"], r["roofline"]["launch_ms_avg"], r["roofline"]["launches_per_step"]))
PY
  tail -1 $out
done
