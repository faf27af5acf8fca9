# round 2: pull threshold (idle lanes before a wave pulls new rays, default 8) on C2 and C3 after the
# one-segment Cartesian step
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log | cut -c1-160; return $rc; }
for t in 8 4 16 24; do run c2_t$t 300 python bench.py --config c2 --no-cpu-baseline --threshold $t || exit 1; done
for t in 8 4 16; do run c3_t$t 300 python bench.py --no-cpu-baseline --threshold $t --steps 3 || exit 1; done
