#!/bin/bash
# Compile-checks the maintainer-side binding (integration/GpuPhotonEngine.cpp) against the reference's own
# headers, the way it would be built inside SKIRTcore. Runs in the build container only (it needs
# /root/reference and the Qt5 headers under /opt/conda); nothing it produces is committed or shipped.
#
# The binding reads state that SKIRT keeps private (the tree node vector, the HG asymmetry parameters, the
# detector arrays, ...), so the maintainer's patch adds `friend class GpuPhotonEngine;` to those classes.
# This script applies exactly that patch to a scratch copy of the affected headers (sed, inserted after
# the class's opening brace) and puts the copy first on the include path. It then compiles the binding to
# an object file with g++ and lists the engine symbols the object needs, which must all be exported by
# skirt_amd/libskirt_amd.so.
#   usage: integration/check_binding.sh [scratch-dir]
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(dirname "$HERE")
REF=${SKIRT_REFERENCE:-/root/reference}
QT=${QT_INCLUDE:-/opt/conda/include/qt}
WORK=${1:-$(mktemp -d)}
mkdir -p "$WORK/overlay"
FRIENDS="DustMix TreeDustGrid TreeNode VoronoiDustGrid SersicGeometry SersicFunction PlummerGeometry ExpDiskGeometry FullInstrument SimpleInstrument FrameInstrument SEDInstrument"
for cls in $FRIENDS; do
  src="$REF/SKIRTcore/$cls.hpp"
  [ -f "$src" ] || { echo "missing $src"; exit 1; }
  # first line that is exactly "{" after the "class <cls>" line
  sed "/^class $cls\b/,/^{/ s/^{\$/{\n    friend class GpuPhotonEngine;  \/\/ MI355X binding (INTEGRATION.md)/" "$src" > "$WORK/overlay/$cls.hpp"
  grep -q "friend class GpuPhotonEngine" "$WORK/overlay/$cls.hpp" || { echo "could not patch $cls"; exit 1; }
done
g++ -std=c++14 -fPIC -O1 -Wall -Wno-deprecated-declarations -DQT_CORE_LIB -DQT_NO_DEBUG \
    -I"$WORK/overlay" -I"$REPO/include" -I"$REPO/integration" \
    -I"$REF/SKIRTcore" -I"$REF/Fundamentals" -I"$REF/Voro" -I"$REF/MPIsupport" \
    -I"$QT" -I"$QT/QtCore" \
    -c "$HERE/GpuPhotonEngine.cpp" -o "$WORK/GpuPhotonEngine.o"
echo "compiled $WORK/GpuPhotonEngine.o"
nm -u "$WORK/GpuPhotonEngine.o" | awk '{print $2}' | grep -E '^skirt_(mcrt|host|sim|rccl)_' | sort -u > "$WORK/needed.txt"
nm -D --defined-only "$REPO/skirt_amd/libskirt_amd.so" | awk '{print $3}' | sort -u > "$WORK/exported.txt"
missing=$(comm -23 "$WORK/needed.txt" "$WORK/exported.txt")
if [ -n "$missing" ]; then echo "symbols missing from libskirt_amd.so: $missing"; exit 1; fi
echo "engine symbols used by the binding: $(tr '\n' ' ' < "$WORK/needed.txt")"
