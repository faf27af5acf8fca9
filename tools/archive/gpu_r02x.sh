# round 2: C4 occupancy / unroll variants of the branch-free Voronoi step
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
run c4_new 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_w2.so run c4_w2 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_u2.so run c4_u2 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_u8.so run c4_u8 300 python bench.py --config c4 --no-cpu-baseline
