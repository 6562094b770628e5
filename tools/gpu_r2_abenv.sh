#!/bin/bash
# Interleaved A/B of one environment knob on a bench workload, in one GPU call:
#   AB_VAR=RAFTSTEP_LIST_STAGE AB_A=1 AB_B=0 WL="--workload C4 --steps 64 --warmup 16" bash tools/gpu_r2_abenv.sh
# RUNTESTS=1 runs the GPU test suite first.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2ab}
mkdir -p $OUT
WL=${WL:---workload C4 --steps 64 --warmup 16}
if [ -n "$RUNTESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
fi
for rep in 1 2; do
  for v in "$AB_A" "$AB_B"; do
    env $AB_VAR=$v timeout -k 10 200 python3 -u bench.py $WL --repeats 3 --no-cpu-baseline > $OUT/ab_${AB_VAR}_${v}_$rep.log 2>&1 || exit 1
  done
done
