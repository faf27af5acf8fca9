# round 2: C5 host-stage timings and kernel trace after the parallel block-sum scan and the lazy dust-Labs
# download; the dust-phase GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c5
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
TAILN=2 run pytest_dust 600 python -u -m pytest tests -m gpu -k "dust or cell_sources or second_run or cs or statistically or per_cell or benchmark_models" -v --timeout 300 --timeout-method thread &&
SKIRT_AMD_PHASE_TIMES=1 TAILN=14 run c5_times 300 python bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5/trace -o run -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c5/trace.log 2>&1 && echo trace ok &&
run c5 300 python bench.py --config c5 --no-cpu-baseline
