# round evidence: smoke + GPU tests + short benches, the default bench line (with the CPU baseline),
# and the rocprofv3 passes of the C3 bench (summarised locally by tools/pmc_traffic.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_check.sh &&
echo "== bench default" && timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log &&
CFG=c3 bash tools/gpu_prof.sh
