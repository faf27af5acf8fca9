# sweep: library variant x trace grid (short C3 runs, each under its own time limit)
# usage: VARIANTS="base h2" GRIDS="0 768 512" bash tools/gpu_sweep2.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
b() { local tag=$1; shift; echo -n "== $tag $* : "; timeout -k 10 200 python bench.py --config ${CFG:-c3} --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/sweep/$tag.log 2>&1 || return 1; python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); ro=r['roofline']; print('%.4g pkt/s  %.1f ms/step  trace %.3f ms x %d  lanes %.3f' % (r['value'], r['ms_per_step'], ro['launch_ms_avg'], ro['launches_per_step'], r['config'].get('lane_use', 0)))" gpurun_out/sweep/$tag.log; }
for v in ${VARIANTS:-base}; do
  for g in ${GRIDS:-0}; do
    if [ $v = base ]; then b ${v}_g$g --trace-grid $g || exit 1
    else SKIRT_AMD_LIB=libskirt_amd_$v.so b ${v}_g$g --trace-grid $g || exit 1; fi
  done
done
