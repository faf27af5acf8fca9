#!/bin/bash
# round-6 GPU call C (tool only): the Voronoi shared entry groups, third build (ballot prefix sum, operands
# through LDS; libskirt_amd_vshare.so, and libskirt_amd_vshareE.so with the shared loads before all own groups):
# Voronoi parity, C4 A/B against the lane-serial default, and one SQ PMC pass each. Logs under gpurun_out/r06c/.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06c; mkdir -p $out
for lib in libskirt_amd_vshare.so libskirt_amd_vshareE.so; do
  SKIRT_AMD_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
      tests/test_gpu_counts.py -k "vor or c4" > $out/vor_tests_$lib.log 2>&1 || { echo "vor tests failed ($lib)"; tail -30 $out/vor_tests_$lib.log; exit 1; }
  echo "$lib: $(tail -1 $out/vor_tests_$lib.log)"
done
c4() {  # tag [lib]
    local tag=$1
    timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline --steps 4 --warmup 1 > $out/$tag.json 2> $out/$tag.err || { echo "FAIL $tag"; exit 1; }
    python - "$out/$tag.json" "$tag" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("%-12s %.4e  ms/step %.1f  trace %.3f ms" % (sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["launch_ms_avg"]), flush=True)
PY
}
for rep in 1 2; do
  c4 c4_serial_$rep
  SKIRT_AMD_LIB=libskirt_amd_vshare.so c4 c4_share_$rep
  SKIRT_AMD_LIB=libskirt_amd_vshareE.so c4 c4_shareE_$rep
done
for v in serial share; do
  lib=libskirt_amd.so; [ $v = share ] && lib=libskirt_amd_vshare.so
  SKIRT_AMD_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
      --output-format csv -d $out/pmc_$v -o run -- python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $out/pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  echo "pmc $v ok"
done
