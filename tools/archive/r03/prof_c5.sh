# round 3: rocprofv3 kernel trace + PMC passes of C5 at its size (1 step) at the final build, then its bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
STEPS=1 CFG=c5 TAG=_full bash tools/gpu_prof.sh > gpurun_out/prof_c5.out 2>&1 && tail -1 gpurun_out/prof_c5.out &&
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 && tail -1 gpurun_out/bench_c5.log | cut -c1-200
