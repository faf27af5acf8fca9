#!/bin/bash
# Builds integration/_build/describe: the maintainer binding (integration/GpuPhotonEngine.cpp, compiled by
# check_binding.sh against the reference's headers with the binding's `friend` patch) linked with the
# reference's own objects (oracle/ref.mk's build, minus its main) and libskirt_amd.so, around
# integration/describe_main.cpp. Build container only (needs /root/reference, Qt5 under /opt/conda and
# oracle/ref.mk's objects); the output stays in the git- and gpurun-ignored integration/_build.
#   usage: integration/build_describe.sh
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(dirname "$HERE")
REF=${SKIRT_REFERENCE:-/root/reference}
QT=${QT:-/opt/conda}
OUT="$HERE/_build"
mkdir -p "$OUT"
make -s -C "$REPO" -f oracle/ref.mk -j8 >/dev/null         # the reference objects (incremental)
bash "$HERE/check_binding.sh" "$OUT" >/dev/null             # GpuPhotonEngine.o against the patched headers
g++ -std=c++14 -fPIC -O1 -Wall -Wno-deprecated-declarations -DQT_CORE_LIB -DQT_NO_DEBUG \
    -I"$OUT/overlay" -I"$REPO/include" -I"$HERE" \
    -I"$REF/SKIRTcore" -I"$REF/Fundamentals" -I"$REF/Voro" -I"$REF/MPIsupport" -I"$REF/Discover" \
    -I"$QT/include/qt" -I"$QT/include/qt/QtCore" \
    -c "$HERE/describe_main.cpp" -o "$OUT/describe_main.o"
REFOBJS=$(ls "$REPO"/oracle/_ref_build/obj/*.o | grep -v '/ref_main\.o$')
# the system libstdc++ first on the run path: libskirt_amd.so needs a newer one than conda's, which Qt's
# libraries would otherwise bring in (the same soname is loaded once)
g++ -o "$OUT/describe" "$OUT/describe_main.o" "$OUT/GpuPhotonEngine.o" $REFOBJS \
    -L"$REPO/skirt_amd" -lskirt_amd "$QT/lib/libQt5Network.so" "$QT/lib/libQt5Core.so" -lpthread \
    -Wl,-rpath,/usr/lib/x86_64-linux-gnu -Wl,-rpath,"$REPO/skirt_amd" -Wl,-rpath,"$QT/lib"
echo "built $OUT/describe"
# FilePaths.cpp:25 looks for the built-in resources in a `dat` folder beside the executable
ln -sfn "$REF/dat" "$OUT/dat"
