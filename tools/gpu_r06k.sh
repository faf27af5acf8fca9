#!/bin/bash
# round-6 GPU call K: the FILL segments' 1 - exp(-dtau) as a degree-9 polynomial (oneMinusExpNeg,
# libskirt_amd_poly.so) against ocml's expm1 (libskirt_amd_base.so). Parity with poly first (same streams, the
# bit-level counts, the attenuation-sensitive thick models), then alternating A/B. Logs under gpurun_out/ab10/.
set -o pipefail
out=gpurun_out/ab10; mkdir -p $out
K="same_streams or replicas or high_index or over_4_gib or aligned or counts or mean_intensity or statistically"
SKIRT_AMD_LIB=libskirt_amd_poly.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_counts.py tests/test_gpu_cartesian.py tests/test_gpu_trees.py -k "$K" > $out/tests.log 2>&1 \
    || { echo "poly tests failed"; tail -30 $out/tests.log; exit 1; }
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
for cfg in c3 c2 c4 c5; do
  for rep in 1 2; do
    for v in poly base; do
      SKIRT_AMD_LIB=libskirt_amd_$v.so run ${cfg}_${v}_$rep --config $cfg
    done
  done
done
