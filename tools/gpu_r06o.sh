#!/bin/bash
# round-6 GPU call O: the Voronoi walk's Labs drain as two round-robin drain instructions per step (drainStep2,
# libskirt_amd_vd2.so) instead of a full drain behind a branch when a buffer might overflow (base). Voronoi
# parity with vd2 first, then alternating C4 benches. Logs under gpurun_out/ab14/.
set -o pipefail
out=gpurun_out/ab14; mkdir -p $out
SKIRT_AMD_LIB=libskirt_amd_vd2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_counts.py tests/test_gpu_setup.py -k "vor or c4" > $out/tests.log 2>&1 \
    || { echo "vd2 tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
run() {
    local tag=$1; shift
    timeout -k 10 170 python -u bench.py --no-cpu-baseline --steps 4 --warmup 1 "$@" > $out/$tag.json 2> $out/$tag.err || { echo "FAIL $tag"; exit 1; }
    python - "$out/$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
f = d["roofline"]
print("%-14s %.4e  ms/step %.1f  trace %.3f ms x %.1f  adds/req %.3f  atomic %.3f" % (sys.argv[2], d["value"], d["ms_per_step"],
      f["launch_ms_avg"], f["launches_per_step"], f["labs_adds_per_request"], f["atomic_frac"]), flush=True)
PY
}
for rep in 1 2 3; do
  for v in vd2 base; do SKIRT_AMD_LIB=libskirt_amd_$v.so run c4_${v}_$rep --config c4; done
done
