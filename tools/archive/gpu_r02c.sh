# round 2: the parity file alone (C5-shape models, per-cell chi^2, run-twice) with the outlier log
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers.jsonl
rm -f $SKIRT_PARITY_LOG
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log; return $rc; }
TAILN=8 run pytest_parity 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 300 --timeout-method thread &&
run bench_c5 300 python bench.py --config c5 --no-cpu-baseline
