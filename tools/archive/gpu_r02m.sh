# round 2: full-size model parity (two-tier outlier criterion); leaf-map step checking the estimate
# against the found leaf's faces (libskirt_amd_faces.so): octree parity tests and the C3/C5 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers_bench.jsonl
rm -f $SKIRT_PARITY_LOG
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
TAILN=2 run pytest_bench_models 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -k benchmark_models -v -s --timeout 600 --timeout-method thread &&
SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers_faces.jsonl SKIRT_AMD_LIB=libskirt_amd_faces.so TAILN=2 run pytest_faces 900 python -u -m pytest tests -m gpu -k "oct or leaf_map or benchmark_models or tree" -v -s --timeout 600 --timeout-method thread &&
run c3 300 python bench.py --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_faces.so run c3_faces 300 python bench.py --no-cpu-baseline &&
run c5 300 python bench.py --config c5 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_faces.so run c5_faces 300 python bench.py --config c5 --no-cpu-baseline
