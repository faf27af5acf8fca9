set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/smoke.log
echo "== pytest gpu"; timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "rc=$?"; tail -15 gpurun_out/pytest_gpu.log
echo "== bench c3"; timeout -k 10 400 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1; echo "rc=$?"; tail -1 gpurun_out/bench_c3.log
echo "== bench c2"; timeout -k 10 300 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1; echo "rc=$?"; tail -1 gpurun_out/bench_c2.log
