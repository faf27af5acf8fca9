#!/bin/bash
# round-6 GPU call N: an explicit vmcnt(0) at the end of the trace waves' pull block (libskirt_amd_pw.so), so that
# the steps after a while-iteration without a pull no longer wait with vmcnt(0) (i.e. for the drain's atomic) at
# the join; against the current build (base). Parity with pw first. Logs under gpurun_out/ab13/.
set -o pipefail
out=gpurun_out/ab13; mkdir -p $out
SKIRT_AMD_LIB=libskirt_amd_pw.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_cartesian.py -k "same_streams" > $out/tests.log 2>&1 \
    || { echo "pw tests failed"; tail -30 $out/tests.log; exit 1; }
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
for cfg in c3 c2 c5 c4; do
  for rep in 1 2; do
    for v in pw base; do
      SKIRT_AMD_LIB=libskirt_amd_$v.so run ${cfg}_${v}_$rep --config $cfg
    done
  done
done
