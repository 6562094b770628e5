#!/bin/bash
# Round 2 A/B of the general kernel on C4: variants "name:lib:general:slow_every"
# (lib "" = the in-tree build; general "lane" = one-lane-per-group kernel).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2ab}
mkdir -p $OUT
WL=${WL:-C4}
for v in $VARIANTS; do
  IFS=: read -r name lib gen se <<< "$v"
  env ${lib:+RAFTSTEP_LIB=$lib} ${gen:+RAFTSTEP_GENERAL=$gen} RAFTSTEP_SLOW_EVERY=$se \
    timeout -k 10 300 python3 -u bench.py --workload $WL --steps ${STEPS:-64} --warmup 16 --repeats 3 --no-cpu-baseline \
    > $OUT/$name.log 2>&1 || exit 1
done
