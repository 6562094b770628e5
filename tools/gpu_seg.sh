#!/bin/bash
# Parity suite, fast-kernel drift probe, then an interleaved C4 A/B against tools/ab_libs/head.so.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/ablib.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/c4_probe.py c4 r7_raft_steady_iso c4_noiso > $OUT/probe_seg.log 2>&1 || exit 1
for i in 1 2; do
  for L in tools/ab_libs/${ALIB:-head}.so raft-sample_amd/lib/libraftstep.so; do
    echo "LIB $L" >> $OUT/ablib.log
    RAFTSTEP_LIB=$L timeout -k 10 200 python -u bench.py --workload C4 --steps 100 --warmup 16 --no-cpu-baseline >> $OUT/ablib.log 2>&1 || exit 1
  done
done
