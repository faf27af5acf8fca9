# round 3: the neighbour-parallel drain step against the lane-serial bounds (debug build prints mismatches)
set -o pipefail
cd $GRAFT_REPO_ROOT
SKIRT_AMD_LIB=libskirt_amd_dbg.so timeout -k 10 100 python -u -m pytest -x -v -s --timeout 80 --timeout-method thread -m gpu \
    tests/test_gpu_counts.py -k "vor_pan" > gpurun_out/wdbg_dbg.log 2>&1; rc=$?
head -60 gpurun_out/wdbg_dbg.log; echo "rc=$rc"
exit $rc
