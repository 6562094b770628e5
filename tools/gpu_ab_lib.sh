#!/bin/bash
# A/B of two library builds (RAFTSTEP_LIB) on C2 at 1M and 4M groups, interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/ablib.log
for i in 1 2; do
  for L in tools/ab_libs/${ALIB:-pre_layout}.so raft-sample_amd/lib/libraftstep.so; do
    echo "LIB $L" >> $OUT/ablib.log
    RAFTSTEP_LIB=$L timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline >> $OUT/ablib.log 2>&1 || exit 1
    RAFTSTEP_LIB=$L timeout -k 10 120 python -u bench.py --groups-per-gpu 4194304 --steps 100 --warmup 10 --no-cpu-baseline >> $OUT/ablib.log 2>&1 || exit 1
  done
done
