# round 2: compact Voronoi step (16-byte neighbour entries with float offsets, exact winner): Voronoi
# same-stream parity (bitwise paths), then C4 bench lines at 16 (default) and 8 entries per load round
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers_vor.jsonl
rm -f $SKIRT_PARITY_LOG
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-300; return $rc; }
TAILN=12 run pytest_vor 600 python -u -m pytest tests -m gpu -k "vor" -v -s --timeout 300 --timeout-method thread &&
run c4_u16 300 python bench.py --config c4 --no-cpu-baseline &&
SKIRT_AMD_LIB=libskirt_amd_vu8.so run c4_u8 300 python bench.py --config c4 --no-cpu-baseline
