#!/bin/bash
# C4 throughput vs general-kernel window (RAFTSTEP_SLOW_EVERY).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/c4_se.log
for se in ${SES:-8 1 2 4 16 8}; do
  echo "SE $se" >> $OUT/c4_se.log
  RAFTSTEP_SLOW_EVERY=$se timeout -k 10 200 python -u bench.py --workload C4 --steps 96 --warmup 16 --no-cpu-baseline >> $OUT/c4_se.log 2>&1 || exit 1
done
