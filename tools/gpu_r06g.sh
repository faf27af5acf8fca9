#!/bin/bash
# round-6 GPU call G: rocprofv3 kernel-trace + PMC passes of the C2, C4 and C5 benches at the final
# build (tools/gpu_prof.sh), so that every config's profiles/pmc_<cfg>.json is of this round's engine.
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in c2 c4 c5; do
  CFG=$cfg STEPS=${STEPS:-5} bash tools/gpu_prof.sh > gpurun_out/prof_$cfg.log 2>&1 || { echo "prof $cfg failed"; tail -20 gpurun_out/prof_$cfg.log; exit 1; }
  echo "prof $cfg ok"
done
