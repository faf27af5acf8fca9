# round 3: rocprofv3 kernel trace + PMC passes of C4 and C2 at their configurations' sizes (1 step), then
# their bench lines with the refreshed per-launch traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
STEPS=1 CFG=c4 bash tools/gpu_prof.sh > gpurun_out/prof_c4.out 2>&1 && tail -1 gpurun_out/prof_c4.out &&
STEPS=1 CFG=c2 bash tools/gpu_prof.sh > gpurun_out/prof_c2.out 2>&1 && tail -1 gpurun_out/prof_c2.out &&
python tools/pmc_traffic.py c4 r03 > /dev/null && python tools/pmc_traffic.py c2 r03 > /dev/null &&
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 && tail -1 gpurun_out/bench_c4.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 && tail -1 gpurun_out/bench_c2.log | cut -c1-200 &&
cp profiles/pmc_c4.json profiles/pmc_c2.json profiles/r03_rocprof_c4.txt profiles/r03_rocprof_c2.txt profiles/r03_rocprof_c4_kernel_stats.csv profiles/r03_rocprof_c2_kernel_stats.csv gpurun_out/
