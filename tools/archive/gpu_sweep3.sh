# sweep: slots in flight and ray-pull threshold on C3 (short runs, each under its own time limit)
# usage: SLOTS="2097152 4194304" THRESH="0 4 16" bash tools/gpu_sweep3.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep3
b() { local tag=$1; shift; echo -n "== $tag $* : "; timeout -k 10 200 python bench.py --config ${CFG:-c3} --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/sweep3/$tag.log 2>&1 || return 1; python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); ro=r['roofline']; print('%.4g pkt/s  %.1f ms/step  trace %.3f ms x %d  lanes %.3f' % (r['value'], r['ms_per_step'], ro['launch_ms_avg'], ro['launches_per_step'], r['config'].get('lane_use', 0)))" gpurun_out/sweep3/$tag.log; }
for s in ${SLOTS:-0}; do
  for t in ${THRESH:-0}; do
    b s${s}_t$t --slots $s --threshold $t || exit 1
  done
done
