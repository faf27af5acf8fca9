# round 3: per-wave timeline of a C3 stellar phase (SKIRT_EXPERIMENT_TIMELINE build) beside the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r03_sharded.log 2>&1; echo "sharded rc=$?"; tail -4 gpurun_out/r03_sharded.log
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_c3_base.log 2>&1 || { echo FAIL base; tail -5 gpurun_out/r03_c3_base.log; exit 1; }
tail -c 600 gpurun_out/r03_c3_base.log
for cfg in ${CFGS:-c3}; do
SKIRT_AMD_LIB=libskirt_amd_tl.so SKIRT_AMD_TIMELINE_OUT=gpurun_out/tl_$cfg.bin timeout -k 10 300 python bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03_${cfg}_tl.log 2>&1 || { echo FAIL tl $cfg; tail -5 gpurun_out/r03_${cfg}_tl.log; exit 1; }
python tools/timeline_waves.py gpurun_out/tl_$cfg.bin > gpurun_out/tl_$cfg.txt && tail -3 gpurun_out/tl_$cfg.txt
done
