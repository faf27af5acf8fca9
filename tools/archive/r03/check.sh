# round 3: GPU tests touched this round (counters, crossed histogram, thick-model cause, reducers), then
# C3/C4 benches of the build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/check.txt
: > $out
export SKIRT_PARITY_LOG=gpurun_out/parity_outliers.jsonl
rm -f $SKIRT_PARITY_LOG
timeout -k 10 700 python -u -m pytest tests/test_gpu_counts.py tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -v -k "${TESTK:-counts or crossed or same_streams or two_ranks}" --timeout 240 --timeout-method thread > gpurun_out/check_tests.log 2>&1
echo "tests rc=$?" | tee -a $out; grep -E "passed|failed" gpurun_out/check_tests.log | tail -3 | tee -a $out
for cfg in c3 c4; do
  timeout -k 10 200 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/check_$cfg.log 2>&1 || { echo "FAIL $cfg"; tail -5 gpurun_out/check_$cfg.log; exit 1; }
  python - $cfg gpurun_out/check_$cfg.log >> $out <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("%-6s %.4e pkt/s  %.1f ms/step  trace %.3f ms x %d  (%s WG/CU)" % (sys.argv[1], r["value"], r["ms_per_step"], r["roofline"]["launch_ms_avg"], r["roofline"]["launches_per_step"], r["config"].get("trace_blocks_per_cu")))
PY
  tail -1 $out
done
if [ -n "$TL" ]; then
  SKIRT_AMD_LIB=libskirt_amd_tl.so SKIRT_AMD_TIMELINE_OUT=gpurun_out/tl_check.bin timeout -k 10 200 python bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tl_check.log 2>&1 || { echo "FAIL tl"; tail -5 gpurun_out/tl_check.log; exit 1; }
  python tools/timeline_waves.py gpurun_out/tl_check.bin > gpurun_out/tl_check.txt && tail -2 gpurun_out/tl_check.txt | tee -a $out
fi
