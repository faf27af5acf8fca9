# round 3: cellIndex candidate groups of 2 (libskirt_amd_g2.so: 20 VGPRs spilled in the Voronoi event kernel)
# against 4 (the build: 46 spilled) -- C4 at its size, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
one() { SKIRT_AMD_LIB=$1 timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cig2.log 2>&1 || { tail -5 gpurun_out/cig2.log; return 1; }
  echo "$1 $(tail -1 gpurun_out/cig2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.4e pkt/s %.1f ms/step trace %.3f ms" % (d["value"], d["ms_per_step"], d["roofline"]["launch_ms_avg"]))')"; }
for v in libskirt_amd_g2.so libskirt_amd.so libskirt_amd_g2.so libskirt_amd.so libskirt_amd_g2.so libskirt_amd.so; do one $v || exit 1; done
