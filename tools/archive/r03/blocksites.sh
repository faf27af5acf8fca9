# round 3: (1) Voronoi block lists with each candidate's exact site inline (one 32-byte record per candidate),
# (2) guide tables for the dust phases' cell draws (locate_clip in a bracket) -- parity of the Voronoi and dust
# phase tests, then C4 A/B (this build, the previous commit = libskirt_amd_base.so, groups of 8 = _g8 without
# (2)) and C5 A/B (this build against the previous commit)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "vor or c4 or c5 or continuous or counts or crossed or convergence or dust or sources or sharded" > gpurun_out/bs_tests.log 2>&1; rc=$?; tail -3 gpurun_out/bs_tests.log; [ $rc = 0 ] || exit $rc
one() { SKIRT_AMD_LIB=$1 timeout -k 10 200 python bench.py --config $2 --steps $3 --warmup 1 --no-cpu-baseline > gpurun_out/bs_b.log 2>&1 || { tail -5 gpurun_out/bs_b.log; return 1; }
  echo "$2 $1 $(tail -1 gpurun_out/bs_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4e pkt/s %.1f ms/step trace %.3f ms" % (d["value"], d["ms_per_step"], d["roofline"]["launch_ms_avg"]))')"; }
for v in libskirt_amd.so libskirt_amd_base.so libskirt_amd_g8.so libskirt_amd.so libskirt_amd_base.so libskirt_amd_g8.so; do one $v c4 2 || exit 1; done
for v in libskirt_amd.so libskirt_amd_base.so libskirt_amd.so libskirt_amd_base.so; do one $v c5 1 || exit 1; done
