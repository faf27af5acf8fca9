# round 3: Cartesian step change A/B (libskirt_amd.so = change, libskirt_amd_base.so = previous commit): same-stream parity incl. the Cartesian tests, then alternating benches
# same-stream parity first, then alternating C3 (and C2, C5) benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "same_streams and not many" tests/test_gpu_cartesian.py > gpurun_out/evab_tests.log 2>&1 || { tail -30 gpurun_out/evab_tests.log; exit 1; }
tail -2 gpurun_out/evab_tests.log
out=gpurun_out/evab.txt
: > $out
for cfg in ${CFGS:-c3}; do
for v in new base new base; do
  lib=libskirt_amd.so; [ $v != new ] && lib=libskirt_amd_$v.so
  SKIRT_AMD_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ea_$v.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/ea_$v.log; exit 1; }
  python - "$cfg $v" gpurun_out/ea_$v.log >> $out <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("%-10s %.4e pkt/s  %.1f ms/step  trace %.3f ms x %d" % (sys.argv[1], r["value"], r["ms_per_step"], r["roofline"]["launch_ms_avg"], r["roofline"]["launches_per_step"]))
PY
  tail -1 $out
done
done
