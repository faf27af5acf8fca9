#!/bin/bash
# Generates the golden reference outputs under tests/golden/ref/ by running the reference SKIRT v7.3
# binary single-threaded (`skirt -t 1` is bit-reproducible).
#
# The binary is built from the reference's own sources by oracle/ref.mk (g++ + the image's Qt moc, no qmake;
# output in the git-ignored oracle/_ref/). Only the resulting output files (data) are committed; no reference
# source or binary enters the repository.
#   usage: make_fixtures.sh [ski seed tag]      (no arguments: every fixture)
#   LIST=1 make_fixtures.sh prints the fixture list ("ski seed tag lean" per line) and runs nothing
#   DEST=<dir> writes elsewhere than tests/golden/ref (the regeneration test compares the two)
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(cd "$HERE/../.." && pwd)
BIN=${SKIRT_REF_BIN:-$REPO/oracle/_ref/skirt}
[ -n "${SKIRT_REF_BIN:-}" ] || [ -n "${LIST:-}" ] || make -s -C "$REPO" -f oracle/ref.mk -j"${JOBS:-8}" >&2
DEST=${DEST:-$HERE/ref}
WORK=$(mktemp -d)
mkdir -p "$DEST"
run() {  # run <ski name under ski/, or a tests/tree_models.py variant> <seed> <tag>
  if [ -n "${LIST:-}" ]; then echo "$1 $2 $3 ${LEAN:-0}"; return; fi
  local ski=$1 seed=$2 tag=$3 src=$HERE/ski/$1.ski
  if [ ! -f "$src" ]; then  # a grid / geometry / mix / output variant of a committed model
    src=$(cd "$REPO/tests" && python3 -c "import sys, tree_models; print(tree_models.write_any(sys.argv[1], sys.argv[2]))" "$ski" "$WORK")
  fi
  sed "s/seed=\"[0-9]*\"/seed=\"$seed\"/" "$src" > "$WORK/$tag.ski"
  (cd "$WORK" && "$BIN" -t 1 -b -o "$WORK" "$WORK/$tag.ski" > "$WORK/$tag.console" 2>&1)
  for f in "$WORK/$tag"_*; do
    case "$f" in
      *_parameters.*|*.console|*_log.txt) ;;
      *) if [ -z "${LEAN:-}" ]; then cp "$f" "$DEST/"; else
           # lean fixtures: the SED (every flux column), the total frames, the per-cell outputs
           case "$f" in *_sed.dat|*_total.fits|*_ds_isrf.dat|*_ds_convergence.dat|*_ds_crossed.dat|*_ds_cellprops.dat)
             case "$tag:$f" in *_out_*:*_ds_isrf.dat) ;; *) cp "$f" "$DEST/" ;; esac ;; esac
         fi ;;
    esac
  done
  grep -h "Finished the stellar emission phase\|Total number of\|Total extinction\|absorbed dust luminosity\|absorbed stellar luminosity\|Convergence\|neighbors per cell\|Computed Voronoi" "$WORK/$tag"_log.txt > "$DEST/${tag}_log_excerpt.txt" || true
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
  # round 4 (the rebuilt reference): what was pinned only through the oracle before. Lean: the SED, the
  # total frames and the per-cell outputs (the _out variants repeat their base model's ISRF, so not that)
  LEAN=1
  run pan_oct_sa 4357 pan_oct_sa_s4357        # C5 shape: octree + self-absorption, fixed cycles
  run pan_oct_sac 4357 pan_oct_sac_s4357      # C5 shape, convergence-driven cycles
  run pan_cart16_cs 4357 pan_cart16_cs_s4357  # continuous scattering (MonteCarloSimulation.cpp:367-434)
  run pan_oct_cs 4357 pan_oct_cs_s4357
  run vor_pan_cs 4357 vor_pan_cs_s4357
  run bin_pan 4357 bin_pan_s4357              # k-d tree, Alternating split directions
  run bin_bary 4357 bin_bary_s4357            # k-d tree, Barycenter split directions
  run bin_full_td 4357 bin_full_td_s4357      # full k-d tree, TopDown search
  run oct_bary 4357 oct_bary_s4357            # barycentric octree
  run oct_pan_td 4357 oct_pan_td_s4357        # octree, TopDown search
  run oct_pan_bk 4357 oct_pan_bk_s4357        # octree, Bookkeeping search
  run oct_bary_bk 4357 oct_bary_bk_s4357
  run cart_odd 4357 cart_odd_s4357            # odd LinMesh bin counts
  run cart_pow 4357 cart_pow_s4357            # PowMesh / SymPowMesh
  run disk_oct 4357 disk_oct_s4357            # ExpDiskGeometry stars and dust
  run disk_cart 4357 disk_cart_s4357
  run bulge_oct 4357 bulge_oct_s4357          # SersicGeometry stars
  run sersic_cart 4357 sersic_cart_s4357      # SersicGeometry dust
  run point_oct 4357 point_oct_s4357          # PointGeometry
  run zubko_cart 4357 zubko_cart_s4357        # MeanZubkoDustMix
  run draineli_cart 4357 draineli_cart_s4357  # DraineLiDustMix
  run pan_oct_out 4357 pan_oct_out_s4357      # ds_convergence, ds_crossed, ds_cellprops
  run pan_cart16_out 4357 pan_cart16_out_s4357
  run vor_pan_out 4357 vor_pan_out_s4357
  run bbody_cart 4357 bbody_cart_s4357        # BlackBodySED
  run quasar_cart 4357 quasar_cart_s4357      # QuasarSED
  run faceon_cart 4357 faceon_cart_s4357      # dust normalized by face-on optical depth
  run edgeon_cart 4357 edgeon_cart_s4357      # ... edge-on optical depth
  run radial_cart 4357 radial_cart_s4357      # ... radial optical depth
  LEAN=
}
if [ $# -ge 3 ]; then LEAN=${4#0}; run "$1" "$2" "$3"; else all; fi
rm -rf "$WORK"
