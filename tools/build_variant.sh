#!/bin/bash
# build a tuning variant of the engine: tools/build_variant.sh TAG [extra hipcc flags...]
# -> skirt_amd/libskirt_amd_TAG.so (select with SKIRT_AMD_LIB=libskirt_amd_TAG.so)
set -e
tag=$1; shift
cd "$(dirname "$0")/../skirt_amd/csrc"
HOST="build/xml.o build/units.o build/build.o build/outputs.o build/dustemission.o build/voronoi.o build/sim.o build/rccl_reducer.o build/describe.o build/voronoi_cells.o"
make -s $HOST
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -ffp-contract=off -mllvm -disable-machine-licm "$@" \
    -c -o build/engine_$tag.o ${SRC:-device/engine.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libskirt_amd_$tag.so build/engine_$tag.o \
    $HOST -L/opt/rocm/lib -lrccl -ldl -lpthread
