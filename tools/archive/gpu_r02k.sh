# round 2 experiment: distinct 64-byte lines and addresses among each wave's buffered Labs adds on C3
# (libskirt_amd_linecount.so, SKIRT_EXPERIMENT_LINE_COUNT): the headroom of a per-wave merge of the adds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
run c3_ref 300 python bench.py --no-cpu-baseline --packets-per-lambda 200000 --steps 1 --warmup 0 &&
SKIRT_AMD_LIB=libskirt_amd_linecount.so run c3_linecount 600 python bench.py --no-cpu-baseline --packets-per-lambda 200000 --steps 1 --warmup 0
