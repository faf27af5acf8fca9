#!/bin/bash
# round-6 GPU call F (tool only): the event kernel at 4 waves per SIMD, 4 blocks per CU (libskirt_amd_e4.so;
# 6-7 VGPRs spilled) against the default (3 waves by its registers, 3 blocks per CU) on C3 and C2.
set -o pipefail
out=gpurun_out/r06f; mkdir -p $out
SKIRT_AMD_LIB=libskirt_amd_e4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "same_streams and not vor and not c4" > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
echo "e4: $(tail -1 $out/tests.log)"
run() {  # tag lib cfg
    SKIRT_AMD_LIB=$2 timeout -k 10 200 python -u bench.py --config $3 --no-cpu-baseline --steps 4 --warmup 1 > $out/$1.json 2> $out/$1.err || { echo "FAIL $1"; exit 1; }
    python - "$out/$1.json" "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
f = d["roofline"]
print("%-16s %.4e  ms/step %.1f  trace %.3f ms x %.0f" % (sys.argv[2], d["value"], d["ms_per_step"], f["launch_ms_avg"], f["launches_per_step"]), flush=True)
PY
}
for cfg in c3 c2; do
  for rep in 1 2; do
    run ${cfg}_base_$rep libskirt_amd.so $cfg
    run ${cfg}_e4_$rep libskirt_amd_e4.so $cfg
  done
done
