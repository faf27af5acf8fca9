# round 3 final check at the head: smoke, the whole GPU suite, the default bench (C3 + CPU baseline), C2 / C4 / C5
# lines, then the C4 and C5 rocprof passes (kernel trace + PMC) at their sizes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-260; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
TAILN=3 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
run bench_default 600 python bench.py &&
run bench_c2 300 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline &&
run bench_c4 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline &&
run bench_c5 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline &&
STEPS=1 CFG=c4 bash tools/gpu_prof.sh > gpurun_out/prof_c4.out 2>&1 && tail -1 gpurun_out/prof_c4.out &&
python tools/pmc_traffic.py c4 r03 > /dev/null && cp profiles/pmc_c4.json profiles/r03_rocprof_c4.txt profiles/r03_rocprof_c4_kernel_stats.csv gpurun_out/
