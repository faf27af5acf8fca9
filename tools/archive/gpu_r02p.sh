# round 2: Voronoi bound variants on C4: default, FMA contraction in the bounds (ct), two-pass candidate
# masks (tp, tp8 with 8 entries per round), both (tpc); the Voronoi parity tests on tp and tpc
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-160; return $rc; }
run c4 300 python bench.py --config c4 --no-cpu-baseline &&
for v in ct tp tp8 tpc; do SKIRT_AMD_LIB=libskirt_amd_$v.so run c4_$v 300 python bench.py --config c4 --no-cpu-baseline || exit 1; done &&
for v in tp tpc; do SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_$v.jsonl SKIRT_AMD_LIB=libskirt_amd_$v.so TAILN=2 run pytest_$v 600 python -u -m pytest tests -m gpu -k "vor" -v --timeout 600 --timeout-method thread || exit 1; done
