# round 3: Voronoi origin-cell cache in the event kernel -- Voronoi parity tests, then C4 at full size
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "vor or c4 or continuous or counts or crossed or convergence" > gpurun_out/vcell_tests.log 2>&1; rc=$?; tail -3 gpurun_out/vcell_tests.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/vcell_c4_$i.log 2>&1 || { tail -5 gpurun_out/vcell_c4_$i.log; exit 1; }
tail -1 gpurun_out/vcell_c4_$i.log | cut -c1-300
done
SKIRT_AMD_LIB=libskirt_amd_tl.so SKIRT_AMD_TIMELINE_OUT=gpurun_out/tl_c4vc.bin timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tl_c4vc.log 2>&1 && python tools/timeline_waves.py gpurun_out/tl_c4vc.bin > gpurun_out/tl_c4vc.txt && tail -3 gpurun_out/tl_c4vc.txt
