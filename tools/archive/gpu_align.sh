# Labs line alignment experiment: GPU parity tests, then C3 with and without aligned sibling groups
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log; return $rc; }
TAILN=6 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
run bench_c3_align 400 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline &&
SKIRT_AMD_CELL_ALIGN=0 run bench_c3_noalign 400 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline
