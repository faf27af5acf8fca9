#!/bin/bash
# Reference outputs for the BASELINE benchmark models (benchmarks/c{2,3,4,5}*.ski) at 1e3 packages per
# wavelength, written by the reference SKIRT v7.3 rebuilt from its own sources (oracle/ref.mk), single-threaded
# (`skirt -t 1`, bit-reproducible). The convergence, cells-crossed and cell-property outputs are switched on.
# Small files are kept whole, the frames and ds_cellprops as digests (bench_digest.py); only these output
# data enter the repository (tests/golden/ref/bench/), never a reference source or binary.
#   usage: make_bench_fixtures.sh [c3_oct128 ...]   (no arguments: all four)
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(cd "$HERE/../.." && pwd)
BIN=${SKIRT_REF_BIN:-$REPO/oracle/_ref/skirt}
[ -n "${SKIRT_REF_BIN:-}" ] || make -s -C "$REPO" -f oracle/ref.mk -j"${JOBS:-8}" >&2
DEST=${DEST:-$HERE/ref/bench}
WORK=$(mktemp -d)
mkdir -p "$DEST"
models=${*:-c2_cart64 c3_oct128 c4_vor1e5 c5_oct128_sa}
for m in $models; do
  tag=${m}_p1e3
  # 1e3 packages per wavelength, the diagnostic outputs on
  python3 "$HERE/bench_ski.py" "$REPO/benchmarks/$m.ski" > "$WORK/$tag.ski"
  (cd "$WORK" && "$BIN" -t 1 -b -o "$WORK" "$WORK/$tag.ski" > "$WORK/$tag.console" 2>&1)
  for f in "$WORK/$tag"_*; do
    case "$f" in
      *_sed.dat|*_ds_convergence.dat|*_ds_crossed.dat) cp "$f" "$DEST/" ;;
    esac
  done
  python3 "$HERE/bench_digest.py" "$WORK" "$tag" > "$DEST/${tag}_digest.json"
  # the log's statements about the grid (its cell count) and the phases, without the output paths
  grep -h "Finished the stellar emission phase\|Total number of\|Total extinction\|absorbed dust luminosity\|absorbed stellar luminosity\|Convergence\|neighbors per cell\|Computed Voronoi\|cells\|nodes" "$WORK/$tag"_log.txt \
    | grep -v "Writing\|Reading" > "$DEST/${tag}_log_excerpt.txt" || true
done
rm -rf "$WORK"
