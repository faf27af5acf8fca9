# round 2: LDS budget against the device limit (detect-kernel SED copies 8/4/2/1/0, device cell sources
# beyond 64 wavelengths): the parity file, then the C3 and C5 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export SKIRT_PARITY_LOG=$PWD/gpurun_out/parity_outliers.jsonl
rm -f $SKIRT_PARITY_LOG
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-300; return $rc; }
python -c "import torch; p=torch.cuda.get_device_properties(0); print('device', p.name, 'shared_memory_per_block', getattr(p, 'shared_memory_per_block', None), 'per_mp', getattr(p, 'shared_memory_per_multiprocessor', None))" > gpurun_out/devprops.log 2>&1
cat gpurun_out/devprops.log
TAILN=8 run pytest_parity 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 300 --timeout-method thread &&
run c3 300 python bench.py --no-cpu-baseline &&
run c5 300 python bench.py --config c5 --no-cpu-baseline
