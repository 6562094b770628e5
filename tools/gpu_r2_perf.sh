#!/bin/bash
# Round 2 perf snapshot: C2 (1M, 4M), C4 at general-kernel cadence 8 and 1.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2perf}
mkdir -p $OUT
B="timeout -k 10 300 python3 -u bench.py --warmup 16 --repeats 3 --no-cpu-baseline"
$B --steps 100 > $OUT/c2.log 2>&1 \
&& $B --steps 48 --groups-per-gpu 4194304 > $OUT/c2_4m.log 2>&1 \
&& RAFTSTEP_SLOW_EVERY=8 $B --steps 64 --workload C4 > $OUT/c4_se8.log 2>&1 \
&& RAFTSTEP_SLOW_EVERY=1 $B --steps 64 --workload C4 > $OUT/c4_se1.log 2>&1
