# round 3: Voronoi step with per-entry Cauchy-Schwarz bounds (VorAux): Voronoi parity + counts, then C4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/vor.txt
: > $out
export SKIRT_PARITY_LOG=gpurun_out/parity_outliers.jsonl
rm -f $SKIRT_PARITY_LOG
timeout -k 10 600 python -u -m pytest tests/test_gpu_counts.py tests/test_gpu_parity.py -x -v -k "vor or c4" --timeout 240 --timeout-method thread > gpurun_out/vor_tests.log 2>&1
echo "tests rc=$?" | tee -a $out; grep -E "passed|failed" gpurun_out/vor_tests.log | tail -3 | tee -a $out
grep -q " failed" gpurun_out/vor_tests.log && exit 1
for v in new base new base; do
  lib=libskirt_amd.so; [ $v = base ] && lib=libskirt_amd_base.so
  SKIRT_AMD_LIB=$lib timeout -k 10 200 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/vor_c4_$v.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/vor_c4_$v.log; exit 1; }
  python - "c4 $v" gpurun_out/vor_c4_$v.log >> $out <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("%-10s %.4e pkt/s  %.1f ms/step  trace %.3f ms x %d  lane_use %.3f" % (sys.argv[1], r["value"], r["ms_per_step"], r["roofline"]["launch_ms_avg"], r["roofline"]["launches_per_step"], r["config"]["lane_use"]))
PY
  tail -1 $out
done
