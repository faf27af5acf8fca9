# round 2, second GPU pass: the GPU tests (with the C5-shape octree self-absorption models, the per-cell
# chi^2 against the reference and the outlier log of every same-stream comparison) and the C5 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers.jsonl
rm -f $SKIRT_PARITY_LOG
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log; return $rc; }
TAILN=6 run pytest_gpu 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread &&
run bench_c5 300 python bench.py --config c5 --no-cpu-baseline
