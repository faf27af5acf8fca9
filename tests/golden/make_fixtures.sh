#!/bin/bash
# Generates the golden reference outputs under tests/golden/ref/ by running the reference SKIRT v7.3
# binary single-threaded (`skirt -t 1` is bit-reproducible).
#
# The reference binary is NOT built by this repository: it needs Qt5 + moc + qmake (the reference's own
# build system), which this project treats as unbuildable (DESIGN.md "Oracle"). The binary used here was
# built in the survey container following SURVEY.md Appendix A; point SKIRT_REF_BIN at it. Only the
# resulting output files (data) are committed; no reference source or binary enters the repository.
set -euo pipefail
BIN=${SKIRT_REF_BIN:-/tmp/skirtprobe/release/SKIRTmain/skirt}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$HERE/ref
WORK=$(mktemp -d)
mkdir -p "$OUT"
run() {  # run <ski> <seed> <tag>
  local ski=$1 seed=$2 tag=$3
  sed "s/seed=\"[0-9]*\"/seed=\"$seed\"/" "$HERE/ski/$ski.ski" > "$WORK/$tag.ski"
  (cd "$WORK" && "$BIN" -t 1 -b -o "$WORK" "$WORK/$tag.ski" > "$WORK/$tag.console" 2>&1)
  for f in "$WORK/$tag"_*; do
    case "$f" in
      *_parameters.*|*.console|*_log.txt) ;;
      *) cp "$f" "$OUT/" ;;
    esac
  done
  grep -h "Finished the stellar emission phase\|Total number of\|Total extinction\|absorbed dust luminosity\|absorbed stellar luminosity\|Convergence\|neighbors per cell\|Computed Voronoi" "$WORK/$tag"_log.txt > "$OUT/${tag}_log_excerpt.txt" || true
}
all() {
  run c1_oligo16 4357 c1_oligo16_s4357
  run c1_oligo16 777 c1_oligo16_s777
  run oligo_2comp 1234 oligo_2comp_s1234
  run pan_cart16 4357 pan_cart16_s4357
  run pan_oct 4357 pan_oct_s4357
  run pan_oct 99 pan_oct_s99
  run pan_cart16_sa 4357 pan_cart16_sa_s4357
  run pan_cart16_sac 4357 pan_cart16_sac_s4357
  run vor_oligo 4357 vor_oligo_s4357
  run vor_pan 4357 vor_pan_s4357
}
# usage: make_fixtures.sh [ski seed tag]   (no arguments: every fixture)
if [ $# -eq 3 ]; then run "$1" "$2" "$3"; else all; fi
rm -rf "$WORK"
ls -la "$OUT"
