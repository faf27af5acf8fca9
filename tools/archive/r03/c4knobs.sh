# round 3: C4 runtime knobs -- pull threshold (idle lanes before a wave pulls rays) and slots in flight
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/c4knobs.txt
: > $out
for a in "" "--threshold 1" "--threshold 4" "--threshold 16" "--slots 4194304" "--slots 16777216" ""; do
  timeout -k 10 200 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline $a > gpurun_out/c4k.log 2>&1 || { echo "FAIL $a"; tail -5 gpurun_out/c4k.log; exit 1; }
  python - "c4 [$a]" gpurun_out/c4k.log >> $out <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("%-22s %.4e pkt/s  %.1f ms/step  trace %.3f ms x %d  lane_use %.3f" % (sys.argv[1], r["value"], r["ms_per_step"], r["roofline"]["launch_ms_avg"], r["roofline"]["launches_per_step"], r["config"]["lane_use"]))
PY
  tail -1 $out
done
