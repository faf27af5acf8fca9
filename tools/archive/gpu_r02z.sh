# round 2: the setup's density sampling on the device -- its GPU tests (with the C3 setup times), then
# the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-200; return $rc; }
TAILN=3 run pytest_setup 600 python -u -m pytest tests/test_gpu_setup.py -v -s --timeout 300 --timeout-method thread &&
SKIRT_AMD_SETUP_TIMES=1 TAILN=12 run setup_times 300 python -c "
import skirt_amd as S
print('host'); S.Simulation('benchmarks/c3_oct128.ski')
print('device'); S.Simulation('benchmarks/c3_oct128.ski', setup_device=0)
" &&
TAILN=2 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
