# kernel timeline of a short C3 bench (rocprofv3 --kernel-trace only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/timeline_${CFG:-c3}
mkdir -p $OUT && rm -rf $OUT/*
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --config ${CFG:-c3} --steps 1 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/log.txt 2>&1
