# round 3: the whole GPU suite, then smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/full_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/full_gpu.log
[ $rc -ne 0 ] && { grep -n "FAILED\|Error\|assert" gpurun_out/full_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/smoke.log; exit $rc
