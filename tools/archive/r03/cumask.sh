# round 3: role streams + CU masks. Same-stream parity with two halves on masked streams, then C3 timelines
# and benches over pipeline layouts (SKIRT_AMD_HALVES / SKIRT_AMD_TRACE_CUS / SKIRT_AMD_EVENT_CUS)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/cumask.txt
: > $out
SKIRT_AMD_HALVES=2 SKIRT_AMD_TRACE_CUS=208 SKIRT_AMD_EVENT_CUS=48 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "same_streams and not many" --timeout 120 --timeout-method thread > gpurun_out/cumask_parity.log 2>&1
echo "parity rc=$?" | tee -a $out; tail -2 gpurun_out/cumask_parity.log | tee -a $out
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config ${CFG:-c3} --steps 2 --warmup 1 --no-cpu-baseline $BARGS > gpurun_out/cm_$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/cm_$name.log; return 1; }
  python - $name gpurun_out/cm_$name.log >> $out <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("%-24s %.4e pkt/s  %.1f ms/step  trace %.3f ms x %d" % (sys.argv[1], r["value"], r["ms_per_step"], r["roofline"]["launch_ms_avg"], r["roofline"]["launches_per_step"]))
PY
  tail -1 $out
}
tl() {  # name env...: timeline variant
  local name=$1; shift
  env SKIRT_AMD_LIB=libskirt_amd_tl.so SKIRT_AMD_TIMELINE_OUT=gpurun_out/tl_$name.bin "$@" timeout -k 10 200 python bench.py --config ${CFG:-c3} --steps 1 --warmup 1 --no-cpu-baseline $BARGS > gpurun_out/tl_$name.log 2>&1 || { echo "FAIL tl $name"; tail -5 gpurun_out/tl_$name.log; return 1; }
  python tools/timeline_waves.py gpurun_out/tl_$name.bin > gpurun_out/tl_$name.txt && echo "tl $name: $(tail -1 gpurun_out/tl_$name.txt)" | tee -a $out
}
run base &&
tl serial_208_48 SKIRT_AMD_TRACE_CUS=208 SKIRT_AMD_EVENT_CUS=48 &&
run h2_208_48 SKIRT_AMD_HALVES=2 SKIRT_AMD_TRACE_CUS=208 SKIRT_AMD_EVENT_CUS=48 &&
run h2_224_32 SKIRT_AMD_HALVES=2 SKIRT_AMD_TRACE_CUS=224 SKIRT_AMD_EVENT_CUS=32 &&
run h2_192_64 SKIRT_AMD_HALVES=2 SKIRT_AMD_TRACE_CUS=192 SKIRT_AMD_EVENT_CUS=64 &&
run h2_nomask SKIRT_AMD_HALVES=2 &&
BARGS="--slots 16777216" run h2_208_48_s24 SKIRT_AMD_HALVES=2 SKIRT_AMD_TRACE_CUS=208 SKIRT_AMD_EVENT_CUS=48 &&
tl h2_208_48 SKIRT_AMD_HALVES=2 SKIRT_AMD_TRACE_CUS=208 SKIRT_AMD_EVENT_CUS=48
