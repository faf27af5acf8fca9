# benches of every config (default C3 line with the CPU baseline) and the C3 rocprofv3 passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== bench c4" && timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 && tail -1 gpurun_out/bench_c4.log &&
echo "== bench default" && timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log &&
CFG=c3 bash tools/gpu_prof.sh
