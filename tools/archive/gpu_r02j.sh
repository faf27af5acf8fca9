# round 2: full GPU suite, smoke, the default bench line (C3 with the CPU baseline), C4/C2/C5 lines, then
# the rocprofv3 passes (kernel trace + PMC) of C3 and C4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers.jsonl
rm -f $SKIRT_PARITY_LOG
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
TAILN=3 run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread &&
run bench_default 600 python bench.py &&
run bench_c4 300 python bench.py --config c4 --no-cpu-baseline &&
run bench_c2 300 python bench.py --config c2 --no-cpu-baseline &&
run bench_c5 300 python bench.py --config c5 --no-cpu-baseline &&
CFG=c3 bash tools/gpu_prof.sh > gpurun_out/prof_c3.out 2>&1 && tail -2 gpurun_out/prof_c3.out &&
CFG=c4 bash tools/gpu_prof.sh > gpurun_out/prof_c4.out 2>&1 && tail -2 gpurun_out/prof_c4.out
