#!/bin/bash
# interleaved A/B/C of builds on one workload: ablib/libraftstep_<name>.so for
# each name in LIBS ("cur" = the in-tree build), ROUNDS rounds
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUTDIR:-r3ab3}
mkdir -p $OUT
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in ${LIBS:-cur prev}; do
    if [ $v = cur ]; then unset RAFTSTEP_LIB; else export RAFTSTEP_LIB=$PWD/ablib/libraftstep_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload ${WL:-C4} --steps 20 --warmup 5 --no-cpu-baseline \
      > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit 1
  done
done
