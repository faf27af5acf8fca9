# GPU parity tests + short C3 bench (+ optional extra configs): tools/gpu_quick.sh [c2 c4 c5 ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log; return $rc; }
summ() { python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); ro=r['roofline']; print('%s %.4g pkt/s  %.1f ms/step  trace %.3f ms x %d  adds/req %.3f' % (sys.argv[1], r['value'], r['ms_per_step'], ro['launch_ms_avg'], ro['launches_per_step'], ro.get('labs_adds_per_request', 0)))" $1; }
TAILN=4 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
for c in c3 "$@"; do
  TAILN=0 run bench_$c 400 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline || exit 1
  summ gpurun_out/bench_$c.log
done
