# round 3: Voronoi entries as m = n / |n|^2 -- Voronoi parity tests, then C4 at full size A/B against the
# previous build (libskirt_amd_base.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "vor or c4 or continuous or counts or crossed or convergence" > gpurun_out/recip_tests.log 2>&1; rc=$?; tail -3 gpurun_out/recip_tests.log; [ $rc = 0 ] || exit $rc
for v in libskirt_amd.so libskirt_amd_base.so libskirt_amd.so libskirt_amd_base.so; do
SKIRT_AMD_LIB=$v timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/recip_c4.log 2>&1 || { tail -5 gpurun_out/recip_c4.log; exit 1; }
echo "$v $(tail -1 gpurun_out/recip_c4.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4e pkt/s %.1f ms/step trace %.3f ms" % (d["value"], d["ms_per_step"], d["roofline"]["launch_ms_avg"]))')"
done
