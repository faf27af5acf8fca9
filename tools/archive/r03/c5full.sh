# round 3: C5 at its per-GPU size (5e6 packets per wavelength per rank: stellar + 3 self-absorption cycles +
# dust emission), stage times, then the rocprofv3 kernel trace + PMC passes of the same command
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SKIRT_AMD_PHASE_TIMES=1 timeout -k 10 400 python bench.py --config c5 --packets-per-lambda 5000000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_bench_c5_full.log 2>&1 || { echo FAIL bench; tail -5 gpurun_out/r03_bench_c5_full.log; exit 1; }
tail -c 400 gpurun_out/r03_bench_c5_full.log
CFG=c5 TAG=_full STEPS=1 BENCH_ARGS="--packets-per-lambda 5000000" bash tools/gpu_prof.sh
