# round 2: C5 kernel-trace profile (where the non-trace time of a step goes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5/trace -o run -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c5/trace.log 2>&1 && echo trace ok
find gpurun_out/prof_c5 -name "*stats*"
