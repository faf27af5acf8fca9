#!/bin/bash
# round-6 GPU call J: drain schedules for the carried same-line run (tools/gpu_r06i.sh measured the branchy one):
# s1 = two drains every step (period 8, carry <= 4), s2 = two every step, the second empty when not due (period 12),
# s1c2 = s1 with carry <= 2; against the build before them (base). Parity for s1 (the default of the source) and
# s2 first. Logs under gpurun_out/ab9/.
set -o pipefail
out=gpurun_out/ab9; mkdir -p $out
K="same_streams or replicas or high_index or over_4_gib or aligned or counts"
SKIRT_AMD_LIB=libskirt_amd_s1.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_counts.py tests/test_gpu_cartesian.py -k "$K" > $out/tests_s1.log 2>&1 \
    || { echo "s1 tests failed"; tail -30 $out/tests_s1.log; exit 1; }
tail -1 $out/tests_s1.log
SKIRT_AMD_LIB=libskirt_amd_s2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py -k "benchmark_models or many_wavelengths" > $out/tests_s2.log 2>&1 \
    || { echo "s2 tests failed"; tail -30 $out/tests_s2.log; exit 1; }
tail -1 $out/tests_s2.log
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
    for v in base s1 s2 s1c2; do
      SKIRT_AMD_LIB=libskirt_amd_$v.so run ${cfg}_${v}_$rep --config $cfg
    done
  done
done
