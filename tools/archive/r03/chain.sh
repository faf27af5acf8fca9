# round 3: FILL->WALK chaining in the trace kernel. Same-stream parity (chain on), then benches chain on/off
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/chain.txt
: > $out
export SKIRT_PARITY_LOG=gpurun_out/parity_outliers.jsonl
rm -f $SKIRT_PARITY_LOG
timeout -k 10 900 python -u -m pytest tests/test_gpu_counts.py tests/test_gpu_parity.py -x -v -k "${TESTK:-counts or crossed or same_streams}" --timeout 240 --timeout-method thread > gpurun_out/chain_tests.log 2>&1
echo "tests rc=$?" | tee -a $out; grep -E "passed|failed" gpurun_out/chain_tests.log | tail -3 | tee -a $out
[ -n "$STOP_ON_FAIL" ] && grep -q failed gpurun_out/chain_tests.log && exit 1
for cfg in ${CFGS:-c3 c2 c5}; do
 for ch in 1 0; do
  SKIRT_AMD_CHAIN=$ch timeout -k 10 200 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/chain_${cfg}_$ch.log 2>&1 || { echo "FAIL $cfg $ch"; tail -5 gpurun_out/chain_${cfg}_$ch.log; exit 1; }
  python - "$cfg chain=$ch" gpurun_out/chain_${cfg}_$ch.log >> $out <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("%-12s %.4e pkt/s  %.1f ms/step  trace %.3f ms x %d  it %d" % (sys.argv[1], r["value"], r["ms_per_step"], r["roofline"]["launch_ms_avg"], r["roofline"]["launches_per_step"], r["config"]["iterations"]))
PY
  tail -1 $out
 done
done
SKIRT_AMD_LIB=libskirt_amd_tl.so SKIRT_AMD_TIMELINE_OUT=gpurun_out/tl_chain.bin timeout -k 10 200 python bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tl_chain.log 2>&1 || { echo "FAIL tl"; tail -5 gpurun_out/tl_chain.log; exit 1; }
python tools/timeline_waves.py gpurun_out/tl_chain.bin > gpurun_out/tl_chain.txt && tail -2 gpurun_out/tl_chain.txt | tee -a $out
