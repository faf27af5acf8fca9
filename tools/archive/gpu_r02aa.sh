# round 2: C3 with the Labs atomics skipped (tuning experiment: what the rest of the trace kernel costs)
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
run c3 300 python bench.py --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_noat.so run c3_noat 300 python bench.py --no-cpu-baseline
