# round 2: LLVM scheduling strategies for the engine (tools/build_variant.sh ilp|memc|trk), C3/C2/C4 benches
# interleaved with the default build; stops at the first failing GPU step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/sched_sweep.txt
: > $out
for cfg in c3 c2 c4; do
  for v in base ilp memc trk; do
    lib=libskirt_amd.so; [ $v != base ] && lib=libskirt_amd_$v.so
    SKIRT_AMD_LIB=$lib timeout -k 10 240 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/sched_${cfg}_$v.log 2>&1 || { echo "FAIL $cfg $v"; tail -5 gpurun_out/sched_${cfg}_$v.log; exit 1; }
    python - "$cfg" "$v" gpurun_out/sched_${cfg}_$v.log >> $out <<'EOF'
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
r = json.loads(line)
print("%s %-5s %.4e pkt/s  trace %.3f ms" % (sys.argv[1], sys.argv[2], r["value"], r["roofline"]["launch_ms_avg"]))
EOF
    tail -1 $out
  done
done
