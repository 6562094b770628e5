#!/bin/bash
# Round 2: where C4's general-kernel time goes. Per-launch worklist sizes
# (RAFTSTEP_DEBUG_WORK) next to per-launch kernel durations (rocprofv3
# kernel trace) at general-kernel cadence 8 and 1.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r2c4
mkdir -p $OUT
for se in 8 1; do
  RAFTSTEP_DEBUG_WORK=1 RAFTSTEP_SLOW_EVERY=$se timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_se$se -o run --output-format csv -- python3 -u bench.py --workload C4 --steps 32 --warmup 16 --no-cpu-baseline > $OUT/se$se.log 2>&1 || exit 1
done
RAFTSTEP_SLOW_EVERY=1 timeout -k 10 240 python3 -u bench.py --workload C4 --steps 64 --warmup 16 --no-cpu-baseline > $OUT/bench_se1.log 2>&1 || exit 1
