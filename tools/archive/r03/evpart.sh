# round 3: event-kernel parts (shader cycles of loads/events, claims/launches, reservations, writes) with the
# event kernel alone on 64 CUs (serial) and co-running with the other half's trace on 192 CUs (two halves)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/evpart.txt
: > $out
tl() {  # name env...
  local name=$1; shift
  env SKIRT_AMD_LIB=libskirt_amd_tl.so SKIRT_AMD_TIMELINE_OUT=gpurun_out/tl_$name.bin "$@" timeout -k 10 200 python bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tl_$name.log 2>&1 || { echo "FAIL tl $name"; tail -5 gpurun_out/tl_$name.log; return 1; }
  python tools/timeline_waves.py gpurun_out/tl_$name.bin > gpurun_out/tl_$name.txt && { echo "== $name"; tail -3 gpurun_out/tl_$name.txt; } | tee -a $out
}
tl serial_192_64 SKIRT_AMD_TRACE_CUS=192 SKIRT_AMD_EVENT_CUS=64 &&
tl h2_192_64 SKIRT_AMD_HALVES=2 SKIRT_AMD_TRACE_CUS=192 SKIRT_AMD_EVENT_CUS=64
