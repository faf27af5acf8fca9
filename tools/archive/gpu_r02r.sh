# round 2: continuous scattering with the path count in memory: its tests and the C4/C3 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
TAILN=2 run pytest_cs 600 python -u -m pytest tests -m gpu -k "_cs or vor" -v --timeout 300 --timeout-method thread &&
run c4 300 python bench.py --config c4 --no-cpu-baseline &&
run c3 300 python bench.py --no-cpu-baseline
