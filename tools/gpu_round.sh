# smoke, GPU tests, benches of every config (default C3 line with the CPU baseline), then the C3
# rocprofv3 passes; stops at the first failing GPU step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
TAILN=3 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
run bench_default 600 python bench.py &&
run bench_c2 300 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline &&
run bench_c4 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline &&
run bench_c5 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline &&
CFG=c3 bash tools/gpu_prof.sh
