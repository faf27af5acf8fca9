# round 3: packet slots in flight at the configurations' sizes: 2^23 (default) vs 2^24 (and 2^22) on C3, C2, C5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
one() { timeout -k 10 250 python bench.py --config $1 --steps 2 --warmup 1 --no-cpu-baseline $2 > gpurun_out/slots.log 2>&1 || { tail -5 gpurun_out/slots.log; return 1; }
  echo "$1 [$2] $(tail -1 gpurun_out/slots.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4e pkt/s %.1f ms/step trace %.3f ms x %d" % (d["value"], d["ms_per_step"], d["roofline"]["launch_ms_avg"], d["roofline"]["launches_per_step"]))')"; }
for cfg in c3 c2; do
  for a in "" "--slots 16777216" "" "--slots 16777216" "--slots 4194304"; do one $cfg "$a" || exit 1; done
done
one c5 "" && one c5 "--slots 16777216"
