# round 2, final numbers: smoke, the default bench line (C3 with the CPU baseline), C2 profile passes,
# C5 and C4 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
run bench_default 600 python bench.py &&
run c5 300 python bench.py --config c5 --no-cpu-baseline &&
run c4 300 python bench.py --config c4 --no-cpu-baseline &&
CFG=c2 bash tools/gpu_prof.sh
