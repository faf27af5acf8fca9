# round 2: one segment per Cartesian step (the exit wall chosen first) -- Cartesian GPU tests and C2
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
TAILN=2 run pytest_cart 600 python -u -m pytest tests -m gpu -k "cart or c1 or oligo or c2" -v --timeout 300 --timeout-method thread &&
run c2 300 python bench.py --config c2 --no-cpu-baseline &&
run c2b 300 python bench.py --config c2 --no-cpu-baseline
