# round 2: detect kernel on the aux stream beside the next iteration (SKIRT_DETECT_OVERLAP=1 build,
# tools/build_variant.sh ovl): same-stream parity of the variant, then C3/C2/C5 benches against the default
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/ovl_sweep.txt
: > $out
SKIRT_AMD_LIB=libskirt_amd_ovl.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -k same_streams \
  --timeout 120 --timeout-method thread > gpurun_out/ovl_parity.log 2>&1 || { echo "parity FAIL"; tail -20 gpurun_out/ovl_parity.log; exit 1; }
tail -1 gpurun_out/ovl_parity.log | tee -a $out
for cfg in c3 c2 c5; do
  for v in base ovl base ovl; do
    lib=libskirt_amd.so; [ $v != base ] && lib=libskirt_amd_$v.so
    SKIRT_AMD_LIB=$lib timeout -k 10 240 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/ovl_${cfg}_$v.log 2>&1 || { echo "FAIL $cfg $v"; tail -5 gpurun_out/ovl_${cfg}_$v.log; exit 1; }
    python - "$cfg" "$v" gpurun_out/ovl_${cfg}_$v.log >> $out <<'EOF'
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
r = json.loads(line)
print("%s %-5s %.4e pkt/s  %.1f ms/step  trace %.3f ms" % (sys.argv[1], sys.argv[2], r["value"], r["ms_per_step"], r["roofline"]["launch_ms_avg"]))
EOF
    tail -1 $out
  done
done
