# round 2: grid steps per ray pull (2, 4 = default, 8) on C3, C2 and C4 at the final build
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-160; return $rc; }
for v in "" _s2 _s8; do
  SKIRT_AMD_LIB=libskirt_amd$v.so run c3$v 300 python bench.py --no-cpu-baseline --steps 3 &&
  SKIRT_AMD_LIB=libskirt_amd$v.so run c2$v 300 python bench.py --config c2 --no-cpu-baseline &&
  SKIRT_AMD_LIB=libskirt_amd$v.so run c4$v 300 python bench.py --config c4 --no-cpu-baseline || exit 1
done
