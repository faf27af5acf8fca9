# smoke, then C4 and C2 at their configs' per-GPU sizes (C4: 1e9 packets / 8 GPUs / 25 lambda = 5e6 per
# lambda; C2: 1e8 packets on one GPU / 10 lambda = 1e7 per lambda) beside the current bench sizes, and C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-400; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
run c4_small 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline &&
run c4_full 300 python bench.py --config c4 --packets-per-lambda 5000000 --steps 2 --warmup 1 --no-cpu-baseline &&
run c2_small 300 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline &&
run c2_full 300 python bench.py --config c2 --packets-per-lambda 10000000 --steps 3 --warmup 1 --no-cpu-baseline &&
run c3 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline
