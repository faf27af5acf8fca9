# round 2: 80-byte ray records (reciprocal direction recomputed by the trace kernel): full GPU suite, then
# the C3, C4, C5 and C2 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers.jsonl
rm -f $SKIRT_PARITY_LOG
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-160; return $rc; }
TAILN=2 run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread &&
run c3 300 python bench.py --no-cpu-baseline &&
run c4 300 python bench.py --config c4 --no-cpu-baseline &&
run c5 300 python bench.py --config c5 --no-cpu-baseline &&
run c2 300 python bench.py --config c2 --no-cpu-baseline
