#!/bin/bash
# resource usage (VGPRs, spills, scratch, occupancy) of the engine's kernels matching a pattern:
# tools/kres.sh PATTERN [extra hipcc flags]
pat=$1; shift
cd "$(dirname "$0")/../skirt_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -ffp-contract=off -mllvm -disable-machine-licm "$@" \
    -c -o /tmp/kres.o device/engine.hip -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk -v pat="$pat" '/Function Name:/ {show = ($0 ~ pat); if (show) {n=$0; sub(/.*Function Name: /,"",n); printf "%s", n}} show && /VGPRs:|ScratchSize|Occupancy|VGPRs Spill/ {v=$0; sub(/.*remark: +/,"",v); sub(/ \[-Rpass.*/,"",v); printf " | %s", v} show && /LDS Size/ {print ""}'
