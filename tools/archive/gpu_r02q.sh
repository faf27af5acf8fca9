# round 2: continuous scattering on the device (contKernel + path records): its same-stream tests, the
# full GPU suite, and the C3/C4 lines (the trace kernel carries the path recording)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers.jsonl
rm -f $SKIRT_PARITY_LOG
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
TAILN=12 run pytest_cs 600 python -u -m pytest tests -m gpu -k "_cs" -v -s --timeout 300 --timeout-method thread &&
TAILN=2 run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread &&
run c3 300 python bench.py --no-cpu-baseline &&
run c4 300 python bench.py --config c4 --no-cpu-baseline
