set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=${CFG:-c3}
ARGS="bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline"
OUT=gpurun_out/prof2_$CFG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ARGS > $OUT/trace.log 2>&1 && echo trace ok &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $OUT/sq -o run -- python3 $ARGS > $OUT/sq.log 2>&1 && echo sq ok &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o run -- python3 $ARGS > $OUT/sq2.log 2>&1 && echo sq2 ok &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $ARGS > $OUT/fetch.log 2>&1 && echo fetch ok
