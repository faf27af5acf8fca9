#!/bin/bash
# round-6 A/B runs on one box (tool only): C3 at 2^24 / 2^25 / 2^26 packet slots and without the drain's
# statistics (timing only, libskirt_amd_nostats.so; C2 too) or with the requests
# sampled in one wave of 8 (libskirt_amd_sampled.so), C5 with its pooled dust
# phases admitted in 1, 2 or 4 waves (SKIRT_AMD_POOL_DIV), C4 with the shared entry groups against the lane-serial
# step (libskirt_amd_vshare0.so). Alternating order; logs under gpurun_out/ab6/.
set -o pipefail
out=gpurun_out/ab6; mkdir -p $out
# the Voronoi same-stream tests with the default build first (its shared entry groups)
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_counts.py \
    -k "vor or c4" > $out/vor_tests.log 2>&1 || { echo "vor tests failed"; tail -30 $out/vor_tests.log; exit 1; }
tail -1 $out/vor_tests.log
run() {  # tag, then bench args (env via the caller)
    local tag=$1; shift
    timeout -k 10 170 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 "$@" > $out/$tag.json 2> $out/$tag.err || { echo "FAIL $tag"; exit 1; }
    python - "$out/$tag.json" "$tag" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print("%-14s %.4e  ms/step %.1f  trace %.3f ms x %.1f" % (sys.argv[2], d["value"], d["ms_per_step"],
      d["roofline"]["launch_ms_avg"], d["roofline"]["launches_per_step"]), flush=True)
PY
}
for rep in 1 2; do
  run c3_s24_$rep --config c3
  run c3_s25_$rep --config c3 --slots 33554432
  run c3_s26_$rep --config c3 --slots 67108864
  SKIRT_AMD_LIB=libskirt_amd_nostats.so run c3_nostats_$rep --config c3
  SKIRT_AMD_LIB=libskirt_amd_sampled.so run c3_sampled_$rep --config c3
done
for rep in 1 2; do
  run c2_$rep --config c2
  SKIRT_AMD_LIB=libskirt_amd_nostats.so run c2_nostats_$rep --config c2
  SKIRT_AMD_LIB=libskirt_amd_sampled.so run c2_sampled_$rep --config c2
done
for rep in 1 2; do
  run c4_share_$rep --config c4
  SKIRT_AMD_LIB=libskirt_amd_vshare0.so run c4_serial_$rep --config c4
done
for rep in 1 2; do
  SKIRT_AMD_POOL_DIV=1 run c5_d1_$rep --config c5
  SKIRT_AMD_POOL_DIV=2 run c5_d2_$rep --config c5
  SKIRT_AMD_POOL_DIV=4 run c5_d4_$rep --config c5
done
