#!/bin/bash
# round-6 GPU call I: the carried same-line run at each drain (SKIRT_LABS_CARRY, libskirt_amd_carry.so: a lane
# keeps its trailing run of up to 4 same-line adds for its next drain, drains every 12 steps instead of 16).
# Same-stream parity with it first, then alternating A/B benches against the build before it
# (libskirt_amd_base.so). Logs under gpurun_out/ab8/.
set -o pipefail
out=gpurun_out/ab8; mkdir -p $out
SKIRT_AMD_LIB=libskirt_amd_carry.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_counts.py tests/test_gpu_cartesian.py \
    -k "same_streams or replicas or high_index or over_4_gib or aligned or counts" > $out/tests.log 2>&1 \
    || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
run() {  # tag, then bench args (env via the caller)
    local tag=$1; shift
    timeout -k 10 170 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 "$@" > $out/$tag.json 2> $out/$tag.err || { echo "FAIL $tag"; exit 1; }
    python - "$out/$tag.json" "$tag" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
f = d["roofline"]
print("%-14s %.4e  ms/step %.1f  trace %.3f ms x %.1f  adds/req %.3f  atomic %.3f" % (sys.argv[2], d["value"], d["ms_per_step"],
      f["launch_ms_avg"], f["launches_per_step"], f["labs_adds_per_request"], f["atomic_frac"]), flush=True)
PY
}
for cfg in c3 c2 c5; do
  for rep in 1 2; do
    SKIRT_AMD_LIB=libskirt_amd_carry.so run ${cfg}_carry_$rep --config $cfg
    SKIRT_AMD_LIB=libskirt_amd_base.so run ${cfg}_base_$rep --config $cfg
  done
done
