# tuning sweep: library variants x engine knobs (short runs, each under its own time limit)
# usage: VARIANTS="w4 w5" KNOBS="--threshold 8;--slots 4194304" bash tools/gpu_sweep.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
b() { local tag=$1; shift; echo "== $tag $*"; timeout -k 10 200 python bench.py --config ${CFG:-c3} --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/sweep/$tag.log 2>&1 || return 1; python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.4g pkt/s  %.1f ms/step  kernel %.1f ms  lanes %.3f  iters %d' % (r['value'], r['ms_per_step'], r['phase_ms_avg'], r['config'].get('lane_use', 0), r['config'].get('iterations', 0)))" gpurun_out/sweep/$tag.log; }
b base || exit 1
for v in $VARIANTS; do SKIRT_AMD_LIB=libskirt_amd_$v.so b $v || exit 1; done
IFS=';'; n=0
for k in $KNOBS; do n=$((n+1)); IFS=' '; b knob$n $k || exit 1; IFS=';'; done
