#!/bin/bash
# round-6 GPU call D (tool only): the Cartesian tests (the 4 GiB table at rtol 1e-9 with slivers, the 40-bit
# index path, the 37.6 GB table), the failed-phase / bound-dust-Labs tests, the RCCL tests. gpurun_out/r06d/.
set -o pipefail
out=gpurun_out/r06d; mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_cartesian.py > $out/cartesian.log 2>&1 || { echo "cartesian failed"; tail -40 $out/cartesian.log; exit 1; }
grep -E "PASSED|FAILED|parity|sliver" $out/cartesian.log | tail -20
timeout -k 10 280 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
    -k "failed_phase or bound_after or second_run" > $out/tests.log 2>&1 || { echo "new tests failed"; tail -30 $out/tests.log; exit 1; }
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_rccl.py > $out/tests_rccl.log 2>&1 || { echo "rccl tests failed"; tail -30 $out/tests_rccl.log; exit 1; }
grep -E "PASSED|FAILED" $out/tests.log $out/tests_rccl.log
