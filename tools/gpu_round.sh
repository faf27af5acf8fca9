# One gpurun call of the round's GPU work, by preset (run from the repo root on the GPU box):
#   gpurun -- 'bash tools/gpu_round.sh [preset] [args]'
# presets
#   round            smoke, the whole GPU suite, the default bench (C3 + CPU baseline), C2/C4/C5 lines, C3 rocprof
#   tests [-k EXPR]  the GPU suite (or the tests matching EXPR)
#   bench CFG...     one bench line per config (3 steps, no CPU baseline)
#   n2gloo           bench.py's own N > 1 path: 2 ranks over gloo sharing the GPU, against 1 rank shooting
#                    the same global packets (--digest: the reduced tallies must agree)
#   ab CFG...        A/B of skirt_amd/libskirt_amd.so (the change) against libskirt_amd_base.so (built from
#                    the previous commit by hand or tools/build_variant.sh): same-stream parity, then
#                    alternating benches new/base/new/base (pkt/s, ms/step, trace ms per launch);
#                    AB_NEW / AB_BASE name other builds, AB_NO_TESTS=1 skips the parity step
#   multi CFG...     MULTI_LIBS="tagA tagB" (- = the default library): alternating benches of several builds;
#                    MULTI_TESTS=1 runs the same-stream parity tests on each first
#   envs CFG...      ENV_SETS="-|VAR=1|VAR=2 OTHER=3|-::--slots 16777216": alternating benches of the default
#                    build under environment settings and extra bench.py arguments (after "::")
#   ktrace CFG...    MULTI_LIBS as for multi: per-kernel average times (rocprofv3 kernel trace) of each build
#   prof CFG         rocprofv3 kernel trace + PMC passes of the bench (tools/gpu_prof.sh)
# Every GPU step runs under its own timeout; the first failing step ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-1} gpurun_out/$name.log; return $rc; }
line() {  # line LABEL LOG: the bench line's headline numbers
  python3 - "$1" "$2" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
f = r["roofline"]
print("%-24s %.4e pkt/s  %.1f ms/step  trace %.3f ms x %.0f  frac %.3f  atomic %.3f" % (
    sys.argv[1], r["value"], r["ms_per_step"], f["launch_ms_avg"], f["launches_per_step"], f["frac"], f["atomic_frac"]))
PY
}
preset=${1:-round}; shift || true
case $preset in
round)
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
  TAILN=3 run pytest_gpu 1200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
  run bench_default 600 python bench.py &&
  run bench_c2 300 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline &&
  run bench_c4 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline &&
  run bench_c5 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline &&
  CFG=c3 bash tools/gpu_prof.sh ;;
tests)
  TAILN=5 run pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@" ;;
bench)
  for cfg in "$@"; do
    run bench_$cfg 400 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline && line $cfg gpurun_out/bench_$cfg.log || exit 1
  done ;;
n2gloo)
  # 2 ranks x 1e6 packets per wavelength per rank = the global packets of 1 rank x 2e6
  run bench_n2_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --packets-per-lambda 1000000 --dist-backend gloo --digest &&
  run bench_n1_same_packets 400 python bench.py --steps 2 --warmup 1 --packets-per-lambda 2000000 --digest --no-cpu-baseline &&
  python3 - gpurun_out/bench_n2_gloo.log gpurun_out/bench_n1_same_packets.log <<'PY'
import json, sys
a, b = [json.loads([l for l in open(p) if l.startswith("{")][-1]) for p in sys.argv[1:3]]
da, db = a["tally_digest"], b["tally_digest"]
rel = lambda x, y: abs(x - y) / max(abs(y), 1e-300)
worst = max(rel(x, y) for x, y in zip(da["labs_per_lambda"], db["labs_per_lambda"]))
print("per rank:", a["per_rank"])
print("labs total %.12e vs %.12e (rel %.2e); worst per-lambda rel %.2e" % (da["labs_total"], db["labs_total"], rel(da["labs_total"], db["labs_total"]), worst))
print("SED total %.12e vs %.12e; frame total %.12e vs %.12e" % (da["sed_total"], db["sed_total"], da["frame_total"], db["frame_total"]))
ok = worst < 1e-9 and rel(da["sed_total"], db["sed_total"]) < 1e-9 and rel(da["frame_total"], db["frame_total"]) < 1e-9
print("N=2 (gloo) tallies equal N=1 at the same global packets:", ok)
sys.exit(0 if ok else 1)
PY
  ;;
ab)
  [ -n "${AB_NO_TESTS:-}" ] || TAILN=2 run ab_tests 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
      tests/test_gpu_counts.py -k "same_streams or counts or crossed" || { [ -n "${AB_NO_TESTS:-}" ] || exit 1; }
  out=gpurun_out/ab.txt; : > $out
  for cfg in "${@:-c3}"; do
    for v in new base new base; do
      lib=${AB_NEW:-libskirt_amd.so}; [ $v != new ] && lib=${AB_BASE:-libskirt_amd_base.so}
      SKIRT_AMD_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline \
          > gpurun_out/ab_${cfg}_$v.log 2>&1 || { echo "FAIL $cfg $v"; tail -5 gpurun_out/ab_${cfg}_$v.log; exit 1; }
      line "$cfg $v" gpurun_out/ab_${cfg}_$v.log >> $out; tail -1 $out
    done
  done ;;
multi)
  # MULTI_LIBS="tagA tagB ..." (libskirt_amd_TAG.so; "-" = libskirt_amd.so): same-stream parity of each
  # (MULTI_TESTS=1), then two alternating bench rounds over the libraries per config
  libs=${MULTI_LIBS:?}; out=gpurun_out/multi.txt; : > $out
  libof() { [ "$1" = - ] && echo libskirt_amd.so || echo libskirt_amd_$1.so; }
  if [ -n "${MULTI_TESTS:-}" ]; then
    for t in $libs; do
      SKIRT_AMD_LIB=$(libof $t) TAILN=2 run multi_tests_$t 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
          -m gpu tests/test_gpu_parity.py tests/test_gpu_counts.py -k "same_streams or counts or crossed" || exit 1
    done
  fi
  [ -n "${MULTI_TESTS:-}" ] && [ $# -eq 0 ] && exit 0  # tests only
  for cfg in "${@:-c3}"; do
    v=MULTI_LIBS_$cfg; cl=${!v:-$libs}  # MULTI_LIBS_c4=... : another set for one config
    for rep in 1 2; do
      for t in $cl; do
        SKIRT_AMD_LIB=$(libof $t) timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline \
            > gpurun_out/multi_${cfg}_${t}_$rep.log 2>&1 || { echo "FAIL $cfg $t"; tail -5 gpurun_out/multi_${cfg}_${t}_$rep.log; exit 1; }
        line "$cfg $t" gpurun_out/multi_${cfg}_${t}_$rep.log >> $out; tail -1 $out
      done
    done
  done ;;
envs)
  # ENV_SETS="-|SKIRT_AMD_WALK_BACK=0|..." ("-": none): two alternating bench rounds per config over engine
  # environment settings (gpurun_out/envs.txt)
  out=gpurun_out/envs.txt; : > $out
  IFS='|' read -ra sets <<< "${ENV_SETS:?}"
  for cfg in "${@:-c3}"; do
    for rep in 1 2; do
      for e in "${sets[@]}"; do
        tag=$(echo "$e" | tr -c 'A-Za-z0-9=\n' _)
        envpart=${e%%::*}; argpart=; [[ "$e" == *::* ]] && argpart=${e#*::}
        ( [ "$envpart" != - ] && [ -n "$envpart" ] && export $envpart; timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline $argpart ) \
            > gpurun_out/envs_${cfg}_${tag}_$rep.log 2>&1 || { echo "FAIL $cfg $e"; tail -5 gpurun_out/envs_${cfg}_${tag}_$rep.log; exit 1; }
        line "$cfg $e" gpurun_out/envs_${cfg}_${tag}_$rep.log >> $out; tail -1 $out
      done
    done
  done ;;
ktrace)
  # MULTI_LIBS as for multi: a rocprofv3 kernel trace of one short bench per library and config, the
  # per-kernel averages side by side (gpurun_out/ktrace.txt)
  libs=${MULTI_LIBS:?}; out=gpurun_out/ktrace.txt; : > $out
  libof() { [ "$1" = - ] && echo libskirt_amd.so || echo libskirt_amd_$1.so; }
  for cfg in "${@:-c3}"; do
    v=MULTI_LIBS_$cfg; cl=${!v:-$libs}
    for t in $cl; do
      d=gpurun_out/kt_${cfg}_$t
      SKIRT_AMD_LIB=$(libof $t) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
          python3 bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > $d.log 2>&1 || { echo "FAIL $cfg $t"; tail -5 $d.log; exit 1; }
      python3 - "$cfg $t" $d >> $out <<'PY'
import csv, glob, re, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[2] + "/**/*kernel_stats.csv", recursive=True)[0])))
short = lambda n: re.search(r"\w+Kernel\w*(<[^>]*>)?", n).group(0).replace(" ", "")
parts = ["%s %.3f ms x %s" % (short(r["Name"]), float(r["AverageNs"]) / 1e6, r["Calls"]) for r in rows
         if any(k in r["Name"] for k in ("traceKernel", "eventKernel", "detectKernel", "contKernel"))]
print("%-16s %s" % (sys.argv[1], " | ".join(parts)))
PY
      tail -1 $out
    done
  done ;;
prof)
  CFG=${1:-c3} bash tools/gpu_prof.sh ;;
*) echo "unknown preset $preset"; exit 2 ;;
esac
