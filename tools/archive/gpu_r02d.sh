# round 2: FMA contraction in the device build (-ffp-contract=fast, libskirt_amd_fma.so) against the
# default build: C3 and C4 bench lines, then the same-stream GPU tests on the variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers_fma.jsonl
rm -f $SKIRT_PARITY_LOG
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-400; return $rc; }
run c3_default 300 python bench.py --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_fma.so run c3_fma 300 python bench.py --no-cpu-baseline &&
run c4_default 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_fma.so run c4_fma 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_fma.so TAILN=4 run pytest_fma 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread
