# round 2: kernel trace of C3 with the Labs add log
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_log/trace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_log/trace.log 2>&1 && echo trace ok
