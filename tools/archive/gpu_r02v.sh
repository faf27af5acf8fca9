# round 2: C2 kernel trace (time outside the photon kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2/trace -o run -- python3 bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c2/trace.log 2>&1 && echo trace ok && grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_c2/trace.log
