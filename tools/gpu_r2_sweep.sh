#!/bin/bash
# Sweep one environment knob over values on a bench workload, in one GPU call:
#   SW_VAR=RAFTSTEP_SLOW_EVERY SW_VALS="1 2 4 8" WL="--workload C4 --steps 64 --warmup 16" bash tools/gpu_r2_sweep.sh
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2sw}
mkdir -p $OUT
WL=${WL:---workload C4 --steps 64 --warmup 16}
for v in $SW_VALS; do
  env $SW_VAR=$v timeout -k 10 200 python3 -u bench.py $WL --repeats 3 --no-cpu-baseline > $OUT/sw_${SW_VAR}_$v.log 2>&1 || exit 1
done
