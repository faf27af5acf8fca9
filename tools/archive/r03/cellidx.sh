# round 3: Voronoi cellIndex with grouped candidate loads (2 / 4 / 8 per round) -- parity, then C4 at full size
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "vor or c4 or continuous or counts or crossed or convergence" > gpurun_out/cellidx_tests.log 2>&1; rc=$?; tail -3 gpurun_out/cellidx_tests.log; [ $rc = 0 ] || exit $rc
for v in libskirt_amd.so libskirt_amd_g2.so libskirt_amd_g8.so libskirt_amd.so; do
SKIRT_AMD_LIB=$v timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cellidx_c4.log 2>&1 || { tail -5 gpurun_out/cellidx_c4.log; exit 1; }
echo "$v $(tail -1 gpurun_out/cellidx_c4.log | cut -c80-180)"
done
SKIRT_AMD_LIB=libskirt_amd_tl.so SKIRT_AMD_TIMELINE_OUT=gpurun_out/tl_c4ci.bin timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tl_c4ci.log 2>&1 && python tools/timeline_waves.py gpurun_out/tl_c4ci.bin > gpurun_out/tl_c4ci.txt && tail -3 gpurun_out/tl_c4ci.txt
