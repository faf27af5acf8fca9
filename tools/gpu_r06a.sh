#!/bin/bash
# round-6 GPU call A (tool only): Voronoi parity with the shared entry groups (stepCoop), the C4 A/B against
# the lane-serial build (libskirt_amd_vshare0.so), the packet trace of the 128^3 Cartesian parity difference
# (libskirt_amd_dbgfill.so, tools/parity_trace.py) and the new GPU tests. Logs under gpurun_out/r06a/.
set -o pipefail
out=gpurun_out/r06a; mkdir -p $out
step() { echo "== $1 $(date +%T)"; }
step vor-tests
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_counts.py \
    -k "vor or c4" > $out/vor_tests.log 2>&1 || { echo "vor tests failed"; tail -30 $out/vor_tests.log; exit 1; }
tail -2 $out/vor_tests.log
c4() {  # tag [env...]
    local tag=$1
    timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline --steps 4 --warmup 1 > $out/$tag.json 2> $out/$tag.err || { echo "FAIL $tag"; exit 1; }
    python - "$out/$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("%-12s %.4e  ms/step %.1f  trace %.3f ms" % (sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["launch_ms_avg"]), flush=True)
PY
}
step c4-ab
for rep in 1 2; do
  c4 c4_share_$rep
  SKIRT_AMD_LIB=libskirt_amd_vshare0.so c4 c4_serial_$rep
done
step trace
mkdir -p $out/ptrace
SKIRT_AMD_LIB=libskirt_amd_dbgfill.so timeout -k 10 600 python -u tools/parity_trace.py engine $out/ptrace > $out/ptrace/run.log 2>&1 || { echo "trace failed"; tail $out/ptrace/run.log; exit 1; }
step new-tests
timeout -k 10 280 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
    -k "failed_phase or bound_after or second_run" > $out/tests.log 2>&1 || { echo "new tests failed"; tail -30 $out/tests.log; exit 1; }
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_rccl.py > $out/tests_rccl.log 2>&1 || { echo "rccl tests failed"; tail -30 $out/tests_rccl.log; exit 1; }
grep -E "passed|failed" $out/tests.log $out/tests_rccl.log
step done
