#!/bin/bash
# round-6 GPU call M (tool only): the trace waves' share of cycles in ray pulls (libskirt_amd_diagpull.so:
# clock64 around the pull block; bench's adds/request then reads all cycles / pull cycles), and the pull
# threshold (idle lanes before a wave pulls rays; default 8) at 4, 16, 32. Logs under gpurun_out/ab12/.
set -o pipefail
out=gpurun_out/ab12; mkdir -p $out
run() {  # tag, then bench args (env via the caller)
    local tag=$1; shift
    timeout -k 10 170 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 "$@" > $out/$tag.json 2> $out/$tag.err || { echo "FAIL $tag"; exit 1; }
    python - "$out/$tag.json" "$tag" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
f = d["roofline"]
print("%-14s %.4e  ms/step %.1f  trace %.3f ms x %.1f  adds/req %.3f  atomic %.3f  lane_use %.3f" % (sys.argv[2], d["value"], d["ms_per_step"],
      f["launch_ms_avg"], f["launches_per_step"], f["labs_adds_per_request"], f["atomic_frac"], d["config"]["lane_use"]), flush=True)
PY
}
for cfg in c3 c2 c5; do SKIRT_AMD_LIB=libskirt_amd_diagpull.so run ${cfg}_diag --config $cfg; done
for rep in 1 2; do
  for t in 8 4 16 32; do run c3_t${t}_$rep --config c3 --threshold $t; done
done
for rep in 1 2; do
  for t in 8 16 32; do run c2_t${t}_$rep --config c2 --threshold $t; done
done
