#!/bin/bash
# round-6 GPU call E (tool only): the trace kernel at 4 waves per SIMD (no spills since round 5's register
# cuts) with 8 or 4 buffered Labs adds per lane (libskirt_amd_w4b8.so, _w4b4.so), against the default (3 waves,
# 16 adds): same-stream parity on the tree and Cartesian models, then alternating benches on C3, C2, C5.
set -o pipefail
out=gpurun_out/r06e; mkdir -p $out
for lib in libskirt_amd_w4b8.so libskirt_amd_w4b4.so; do
  SKIRT_AMD_LIB=$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
      -k "same_streams and not vor and not c4" > $out/tests_$lib.log 2>&1 || { echo "tests failed ($lib)"; tail -30 $out/tests_$lib.log; exit 1; }
  echo "$lib: $(tail -1 $out/tests_$lib.log)"
done
run() {  # tag lib cfg
    SKIRT_AMD_LIB=$2 timeout -k 10 200 python -u bench.py --config $3 --no-cpu-baseline --steps 4 --warmup 1 > $out/$1.json 2> $out/$1.err || { echo "FAIL $1"; exit 1; }
    python - "$out/$1.json" "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
f = d["roofline"]
print("%-16s %.4e  ms/step %.1f  trace %.3f ms x %.0f  atomic %.3f  blocks/CU %s" % (sys.argv[2], d["value"], d["ms_per_step"],
      f["launch_ms_avg"], f["launches_per_step"], f["atomic_frac"], d["config"].get("trace_blocks_per_cu")), flush=True)
PY
}
for cfg in c3 c2 c5; do
  for rep in 1 2; do
    run ${cfg}_base_$rep libskirt_amd.so $cfg
    run ${cfg}_w4b8_$rep libskirt_amd_w4b8.so $cfg
    run ${cfg}_w4b4_$rep libskirt_amd_w4b4.so $cfg
  done
done
