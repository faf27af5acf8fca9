# round 2: C4 entries per round (2, 4, 8) at 2 waves/SIMD, and 4 at 3 waves, on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-160; return $rc; }
for v in "" _u2 _u8 _w3; do SKIRT_AMD_LIB=libskirt_amd$v.so run c4$v 300 python bench.py --config c4 --no-cpu-baseline || exit 1; done
