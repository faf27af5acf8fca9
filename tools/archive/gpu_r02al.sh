# round 2: event kernel blocks per CU (SKIRT_AMD_EVENT_BPC, default 2 = the resident limit at 2 waves/SIMD)
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-160; return $rc; }
for b in 2 4 8 1; do SKIRT_AMD_EVENT_BPC=$b run c2_b$b 300 python bench.py --config c2 --no-cpu-baseline || exit 1; done
for b in 2 4; do SKIRT_AMD_EVENT_BPC=$b run c3_b$b 300 python bench.py --no-cpu-baseline --steps 3 || exit 1; done
