#!/bin/bash
# Repeatability: C2 and C4 bench lines, three runs each (separate processes).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/rep.log
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --workload C4 --steps 100 --warmup 16 --no-cpu-baseline >> $OUT/rep.log 2>&1 || exit 1
  timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline >> $OUT/rep.log 2>&1 || exit 1
done
