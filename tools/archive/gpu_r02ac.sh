# round 2: the ray queue split into FILL/WALK rays and peel-offs -- all GPU tests, then C2, C3, C4, C5
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
TAILN=2 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread &&
run c2 300 python bench.py --config c2 --no-cpu-baseline &&
run c3 300 python bench.py --no-cpu-baseline &&
run c4 300 python bench.py --config c4 --no-cpu-baseline &&
run c5 300 python bench.py --config c5 --no-cpu-baseline
