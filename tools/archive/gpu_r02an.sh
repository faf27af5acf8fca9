# round 2: the device-setup tests (including a photon phase after a device setup)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_setup.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_setup.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_setup.log; exit $rc
