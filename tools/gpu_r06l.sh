#!/bin/bash
# round-6 GPU call L: the drain's global-atomic path as a kernel of its own (Tracer GLOBAL; the octree step's
# leaf-map entry then waits with vmcnt(1) instead of vmcnt(0), i.e. no longer for the previous step's Labs
# atomic), with and without the L2-warming load of the leaf after the next (LeafMapGrid::warm). Variants:
# base = HEAD, poly = + polynomial 1 - exp(-x), g = + GLOBAL kernels, gw = + warm. Parity with gw and g first.
set -o pipefail
out=gpurun_out/ab11; mkdir -p $out
K="same_streams or replicas or high_index or over_4_gib or aligned or counts"
SKIRT_AMD_LIB=libskirt_amd_gw.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_counts.py tests/test_gpu_cartesian.py -k "$K" > $out/tests_gw.log 2>&1 \
    || { echo "gw tests failed"; tail -30 $out/tests_gw.log; exit 1; }
tail -1 $out/tests_gw.log
SKIRT_AMD_LIB=libskirt_amd_g.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_cartesian.py -k "benchmark_models or high_index or over_4_gib" > $out/tests_g.log 2>&1 \
    || { echo "g tests failed"; tail -30 $out/tests_g.log; exit 1; }
tail -1 $out/tests_g.log
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
for cfg in c3 c5 c2; do
  for rep in 1 2; do
    for v in base poly g gw; do
      SKIRT_AMD_LIB=libskirt_amd_$v.so run ${cfg}_${v}_$rep --config $cfg
    done
  done
done
for rep in 1 2; do
  for v in poly g; do
    SKIRT_AMD_LIB=libskirt_amd_$v.so run c4_${v}_$rep --config c4
  done
done
