# round 2: branch-free Voronoi bounds (walls as mirror-image bisectors), exact re-evaluation over the
# possible winners only -- Voronoi GPU parity tests, then C4 for the new build and the previous one
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-240; return $rc; }
TAILN=2 run pytest_vor 600 python -u -m pytest tests -m gpu -k "vor" -v --timeout 300 --timeout-method thread &&
run c4_new 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_old.so run c4_old 300 python bench.py --config c4 --no-cpu-baseline &&
run c4_new2 300 python bench.py --config c4 --no-cpu-baseline
