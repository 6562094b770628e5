#!/bin/bash
# Interleaved A/B of library variants on one box: ROUNDS rounds of bench.py
# lines, one per variant per round ("base" = raft-sample_amd/lib, else
# ablib/<name>). Then, with TESTS set, the named tests on each non-base variant.
#   OUTDIR=r4ab VARIANTS="base la32" ARGS="--workload C4" ROUNDS=3 TESTS="tests/test_gpu_fullsize.py" bash tools/gpu_ab.sh
# BUILD="la32:-DRAFTSTEP_LIST_LANES=32 other:-DX" builds those variants on the box first
# (tools/ablib.sh; ablib/ does not travel with the snapshot).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r4ab}
mkdir -p "$OUT"
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fused --extra none"
# a variant is NAME (the library ablib/NAME, "base" = the tree's) or
# LABEL+VAR=VAL[+VAR=VAL...] (the tree's library with those environment knobs)
variant() {   # sets label, lib, envs
  local v=$1
  label=${v%%+*}; envs=""; lib=raft-sample_amd/lib/libraftstep.so
  if [[ "$v" == *+* ]]; then envs=$(echo "${v#*+}" | tr '+' ' ');
  elif [ -f "raft-sample_amd/lib/ab/$v/libraftstep.so" ]; then lib=raft-sample_amd/lib/ab/$v/libraftstep.so;   # (pushed prebuilt)
  elif [ "$v" != base ]; then lib=ablib/$v/libraftstep.so; fi
}
for b in $BUILD; do
  echo "== $(date +%T) build ${b%%:*}" >> "$OUT/progress.log"
  timeout -k 10 600 bash tools/ablib.sh "${b%%:*}" $(echo "${b#*:}" | tr ',' ' ') >> "$OUT/build.log" 2>&1 || { echo "build $b failed"; exit 1; }
done
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in $VARIANTS; do
    variant "$v"
    echo "== $(date +%T) round $r $label" >> "$OUT/progress.log"
    env RAFTSTEP_LIB=$lib $envs timeout -k 10 300 $B $ARGS > "$OUT/${label}_$r.json" 2> "$OUT/${label}_$r.err" || { echo "bench $label failed"; exit 1; }
  done
done
if [ -n "$TESTS" ]; then
  for v in $VARIANTS; do
    [ "$v" = base ] && continue
    variant "$v"
    echo "== $(date +%T) tests $label" >> "$OUT/progress.log"
    env RAFTSTEP_LIB=$lib $envs timeout -k 10 900 python3 -u -m pytest $TESTS -m gpu -x -v --timeout 600 \
      --timeout-method thread > "$OUT/tests_$label.log" 2>&1 || { echo "tests $label failed"; exit 1; }
  done
fi
echo "== $(date +%T) done" >> "$OUT/progress.log"
