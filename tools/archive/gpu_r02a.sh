# round 2, first GPU pass: smoke, GPU tests, the default bench line, and the FETCH_SIZE calibration of
# scattered gathers (tools/gather_bench.hip); stops at the first failing GPU step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
TAILN=3 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread &&
run bench_default 600 python bench.py &&
run gather_plain 120 tools/gather_bench &&
run gather_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/gather_fetch -o run -- tools/gather_bench &&
run gather_trace 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gather_trace -o run -- tools/gather_bench
