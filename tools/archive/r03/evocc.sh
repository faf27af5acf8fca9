# round 3: new counters tests + quick parity, then event-kernel occupancy variants (waves/EU 3, 4) on C3,
# serial and with the CU-split two-half pipeline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/evocc.txt
: > $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_counts.py tests/test_gpu_parity.py -x -v -k "counts or crossed or same_streams" --timeout 200 --timeout-method thread > gpurun_out/evocc_tests.log 2>&1
echo "tests rc=$?" | tee -a $out; grep -E "passed|failed|Error|assert" gpurun_out/evocc_tests.log | tail -8 | tee -a $out
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config ${CFG:-c3} --steps 2 --warmup 1 --no-cpu-baseline $BARGS > gpurun_out/eo_$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/eo_$name.log; return 1; }
  python - $name gpurun_out/eo_$name.log >> $out <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("%-24s %.4e pkt/s  %.1f ms/step  trace %.3f ms x %d" % (sys.argv[1], r["value"], r["ms_per_step"], r["roofline"]["launch_ms_avg"], r["roofline"]["launches_per_step"]))
PY
  tail -1 $out
}
run base &&
run ev3_b3 SKIRT_AMD_LIB=libskirt_amd_ev3.so SKIRT_AMD_EVENT_BPC=3 &&
run ev4_b4 SKIRT_AMD_LIB=libskirt_amd_ev4.so SKIRT_AMD_EVENT_BPC=4 &&
run ev4_b2 SKIRT_AMD_LIB=libskirt_amd_ev4.so SKIRT_AMD_EVENT_BPC=2 &&
run ev4_h2_192_64 SKIRT_AMD_LIB=libskirt_amd_ev4.so SKIRT_AMD_EVENT_BPC=4 SKIRT_AMD_HALVES=2 SKIRT_AMD_TRACE_CUS=192 SKIRT_AMD_EVENT_CUS=64 &&
run ev4_h2_208_48 SKIRT_AMD_LIB=libskirt_amd_ev4.so SKIRT_AMD_EVENT_BPC=4 SKIRT_AMD_HALVES=2 SKIRT_AMD_TRACE_CUS=208 SKIRT_AMD_EVENT_CUS=48 &&
run h2_176_80 SKIRT_AMD_HALVES=2 SKIRT_AMD_TRACE_CUS=176 SKIRT_AMD_EVENT_CUS=80
