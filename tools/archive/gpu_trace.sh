# kernel trace of a short bench run (no counters): per-launch durations for tools/timeline.py
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=${CFG:-c3}
OUT=gpurun_out/trace_$CFG
mkdir -p $OUT && rm -rf $OUT/*
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $OUT/log 2>&1 && tail -1 $OUT/log | cut -c1-200
