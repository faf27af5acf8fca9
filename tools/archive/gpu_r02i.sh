# round 2: compact Voronoi step, unroll 4 at 3 waves per SIMD (default) against 2, 6, and 4 at 4 waves
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-160; return $rc; }
run c4_u4w3 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_u2w3.so run c4_u2w3 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_u6w3.so run c4_u6w3 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_u4w4.so run c4_u4w4 300 python bench.py --config c4 --no-cpu-baseline &&
run c3 300 python bench.py --no-cpu-baseline
