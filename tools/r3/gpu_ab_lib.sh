#!/bin/bash
# interleaved A/B of the current build against ablib/libraftstep_prev.so on
# one workload (bench.py at the driver's protocol), WL / ROUNDS selectable
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${OUTDIR:-r3ablib}
mkdir -p $OUT
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in new prev; do
    if [ $v = prev ]; then export RAFTSTEP_LIB=$PWD/ablib/libraftstep_prev.so; else unset RAFTSTEP_LIB; fi
    timeout -k 10 300 python -u bench.py --workload ${WL:-C4} --steps 20 --warmup 5 --no-cpu-baseline \
      > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit 1
  done
done
