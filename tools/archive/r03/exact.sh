# round 3: exp(-tau) per FILL segment (the reference's form) with the per-step Labs drain (new), against the
# per-step drain alone (sm) and the previous commit (base): same-stream parity (thick models included), then
# C3, C4, C2 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "same_streams and not many" > gpurun_out/exact_tests.log 2>&1 || { tail -40 gpurun_out/exact_tests.log; exit 1; }
tail -2 gpurun_out/exact_tests.log
out=gpurun_out/exact.txt
: > $out
for cfg in c3 c4 c2; do
for v in new sm base new; do
  lib=libskirt_amd.so; [ $v != new ] && lib=libskirt_amd_$v.so
  SKIRT_AMD_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ex_$v.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/ex_$v.log; exit 1; }
  python - "$cfg $v" gpurun_out/ex_$v.log >> $out <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("%-10s %.4e pkt/s  %.1f ms/step  trace %.3f ms x %d" % (sys.argv[1], r["value"], r["ms_per_step"], r["roofline"]["launch_ms_avg"], r["roofline"]["launches_per_step"]))
PY
  tail -1 $out
done
done
