# round 2: the Labs add log (appended by the trace kernel, added into Labs by bucket in LDS) -- GPU tests,
# then every config with the log and C3 without it
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-160; return $rc; }
TAILN=3 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread &&
run c3 300 python bench.py --no-cpu-baseline &&
SKIRT_AMD_LABS_LOG=0 run c3_nolog 300 python bench.py --no-cpu-baseline &&
run c2 300 python bench.py --config c2 --no-cpu-baseline &&
run c5 300 python bench.py --config c5 --no-cpu-baseline &&
run c4 300 python bench.py --config c4 --no-cpu-baseline
