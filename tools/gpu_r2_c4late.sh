#!/bin/bash
# Does C4's tick cost grow with time (ring-phase drift)? The C4 bench line
# early (warm-up 16) and late (warm-up 1000), lane classes late, and HBM
# traffic of the lean / list kernels late (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2c4late}
mkdir -p $OUT
P="timeout -s KILL 120 rocprofv3"
B="python3 -u bench.py --no-cpu-baseline --workload C4"
L="--workload C4 --steps 24 --warmup 1000 --repeats 1 --no-cpu-baseline"
step() { echo "== $(date +%T) $1" >> $OUT/progress.log; }
step early && timeout -k 10 200 $B --steps 64 --warmup 16 --repeats 3 > $OUT/c4_early.log 2>&1 \
&& step late && timeout -k 10 200 $B --steps 64 --warmup 1000 --repeats 3 > $OUT/c4_late.log 2>&1 \
&& step diag && RAFTSTEP_DEBUG_FAST=1 timeout -k 10 200 $B --steps 32 --warmup 1000 --repeats 1 > $OUT/c4_late_diag.log 2>&1 \
&& step pmc && $P --pmc FETCH_SIZE -T -d $OUT/pmc_late_fetch -o p --output-format csv -- python3 -u bench.py $L > $OUT/pmc1.log 2>&1 \
&& $P --pmc WRITE_SIZE -T -d $OUT/pmc_late_write -o p --output-format csv -- python3 -u bench.py $L > $OUT/pmc2.log 2>&1 \
&& step done
