# round 2: 8 Voronoi entries per round as the default -- Voronoi GPU tests and C4
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-160; return $rc; }
TAILN=2 run pytest_vor 600 python -u -m pytest tests -m gpu -k "vor or benchmark_models" -v --timeout 300 --timeout-method thread &&
run c4 300 python bench.py --config c4 --no-cpu-baseline
