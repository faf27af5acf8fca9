# rocprofv3 passes over the C3 bench: kernel trace + stats, then separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; MI355X_MICROARCH.md rocprofv3 PMC slots).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=${CFG:-c3}
ARGS="bench.py --config $CFG --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline $BENCH_ARGS"
OUT=gpurun_out/prof_$CFG${TAG}
mkdir -p $OUT && rm -rf $OUT/* && echo "python3 $ARGS" > $OUT/cmd.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ARGS > $OUT/trace.log 2>&1 && echo trace ok &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $ARGS > $OUT/fetch.log 2>&1 && echo fetch ok &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $ARGS > $OUT/write.log 2>&1 && echo write ok &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $OUT/sq -o run -- python3 $ARGS > $OUT/sq.log 2>&1 && echo sq ok &&
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/tcc -o run -- python3 $ARGS > $OUT/tcc.log 2>&1 && echo tcc ok &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o run -- python3 $ARGS > $OUT/sq2.log 2>&1 && echo sq2 ok
find $OUT -name "*.csv" | head -20
