# tuning sweep on C3: library variants x engine knobs (short runs, each under its own time limit)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
b() { local tag=$1; shift; echo "== $tag $*"; timeout -k 10 200 python bench.py --config ${CFG:-c3} --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/sweep/$tag.log 2>&1 || return 1; python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.4g pkt/s  %.1f ms/step' % (r['value'], r['ms_per_step']))" gpurun_out/sweep/$tag.log; }
b base &&
SKIRT_AMD_LIB=libskirt_amd_w3.so b w3 &&
SKIRT_AMD_LIB=libskirt_amd_w4.so b w4 &&
b thr4 --threshold 4 &&
b thr32 --threshold 32 &&
b thr64 --threshold 64 &&
b slots1M --slots 1048576 &&
b slots4M --slots 4194304 &&
SKIRT_AMD_LEAFMAP=0 b nodes
