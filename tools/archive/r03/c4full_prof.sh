# round 3: C4 at its per-GPU size -- kernel trace (event / trace / detect split) and the per-wave timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_c4full; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1 && echo trace ok &&
find $OUT/trace -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-8 | head -12 &&
SKIRT_AMD_LIB=libskirt_amd_tl.so SKIRT_AMD_TIMELINE_OUT=gpurun_out/tl_c4full.bin timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tl_c4full.log 2>&1 && python tools/timeline_waves.py gpurun_out/tl_c4full.bin > gpurun_out/tl_c4full.txt && tail -3 gpurun_out/tl_c4full.txt
