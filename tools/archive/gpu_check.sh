# smoke, GPU parity tests, short benches; stops at the first failing GPU step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
TAILN=15 run pytest_gpu 900 python -m pytest tests -m gpu -x -q &&
run bench_c3 400 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline &&
run bench_c2 300 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline
