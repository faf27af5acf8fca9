# round 3: WALK rays queued at the top of the ray queue (pulled last) -- same-stream parity, then C3 / C2 / C4
# A/B against event order (SKIRT_AMD_WALK_BACK=0), and the C3 timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "same_streams or counts or crossed or vor or continuous or sharded" > gpurun_out/wb_tests.log 2>&1; rc=$?; tail -3 gpurun_out/wb_tests.log; [ $rc = 0 ] || exit $rc
b() { local tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $BARGS > gpurun_out/wb.log 2>&1 || { tail -5 gpurun_out/wb.log; return 1; }
  echo "$tag $BARGS $(tail -1 gpurun_out/wb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4e pkt/s %.1f ms/step trace %.3f ms x %d" % (d["value"], d["ms_per_step"], d["roofline"]["launch_ms_avg"], d["roofline"]["launches_per_step"]))')"; }
for cfg in c3 c2 c4; do
  BARGS="--config $cfg"
  b back SKIRT_AMD_WALK_BACK=1 && b order SKIRT_AMD_WALK_BACK=0 && b back SKIRT_AMD_WALK_BACK=1 && b order SKIRT_AMD_WALK_BACK=0 || exit 1
done
SKIRT_AMD_LIB=libskirt_amd_tl.so SKIRT_AMD_TIMELINE_OUT=gpurun_out/tl_c3wb.bin timeout -k 10 300 python bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tl_c3wb.log 2>&1 && python tools/timeline_waves.py gpurun_out/tl_c3wb.bin > gpurun_out/tl_c3wb.txt && tail -1 gpurun_out/tl_c3wb.txt
