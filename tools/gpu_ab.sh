#!/bin/bash
# Parity suite, then an interleaved A/B of two library builds (RAFTSTEP_LIB:
# tools/ab_libs/$ALIB.so vs the in-tree build) on the workloads in $WLS.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/ablib.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2; do
  for L in tools/ab_libs/${ALIB:-head}.so raft-sample_amd/lib/libraftstep.so; do
    for W in ${WLS:-C2 C4}; do
      echo "LIB $L" >> $OUT/ablib.log
      RAFTSTEP_LIB=$L timeout -k 10 200 python -u bench.py --workload $W --steps 100 --warmup 16 --no-cpu-baseline >> $OUT/ablib.log 2>&1 || exit 1
    done
  done
done
