# round 2: A/B of the leaf-map face check (libskirt_amd_faces.so) on C3/C5 and of the packed-f32 Voronoi
# bounds (libskirt_amd_packed.so) on C4, then the parity tests of both variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-160; return $rc; }
run c3 300 python bench.py --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_faces.so run c3_faces 300 python bench.py --no-cpu-baseline &&
run c5 300 python bench.py --config c5 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_faces.so run c5_faces 300 python bench.py --config c5 --no-cpu-baseline &&
run c4 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_packed.so run c4_packed 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers_faces.jsonl SKIRT_AMD_LIB=libskirt_amd_faces.so TAILN=2 run pytest_faces 900 python -u -m pytest tests -m gpu -k "oct or leaf_map or benchmark_models or tree" -v -s --timeout 600 --timeout-method thread &&
SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers_packed.jsonl SKIRT_AMD_LIB=libskirt_amd_packed.so TAILN=2 run pytest_packed 900 python -u -m pytest tests -m gpu -k "vor or benchmark_models" -v -s --timeout 600 --timeout-method thread
