# round 2: single-precision bounds in the compact Voronoi step: Voronoi same-stream parity, then C4 at
# unroll 8 (default), 16, 4, and at 3 waves per SIMD (spilling)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers_vor.jsonl
rm -f $SKIRT_PARITY_LOG
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
TAILN=3 run pytest_vor 600 python -u -m pytest tests -m gpu -k "vor" -v -s --timeout 300 --timeout-method thread &&
run c4_u8 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_u16.so run c4_u16 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_u4.so run c4_u4 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_u8w3.so run c4_u8w3 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_u4w3.so run c4_u4w3 300 python bench.py --config c4 --no-cpu-baseline
