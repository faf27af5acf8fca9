# round 2: the event kernel walking every slot while most are active (SKIRT_EVENT_DENSE 6 = above 6/8;
# variants 8 = never, 4 = above half) -- GPU tests, then C3/C2/C5 per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-160; return $rc; }
TAILN=2 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread &&
for v in "" _d8 _d4; do
  SKIRT_AMD_LIB=libskirt_amd$v.so run c3$v 300 python bench.py --no-cpu-baseline &&
  SKIRT_AMD_LIB=libskirt_amd$v.so run c2$v 300 python bench.py --config c2 --no-cpu-baseline &&
  SKIRT_AMD_LIB=libskirt_amd$v.so run c5$v 300 python bench.py --config c5 --no-cpu-baseline || exit 1
done
