#!/bin/bash
# C4 lane-class counters of the two-pass tick (RAFTSTEP_DEBUG_FAST, summed over
# both kernels) and the general kernel's worklist sizes (RAFTSTEP_DEBUG_WORK).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2d}
mkdir -p $OUT
RAFTSTEP_DEBUG_FAST=1 timeout -k 10 200 python3 -u bench.py --workload C4 --steps 32 --warmup 16 --repeats 1 --no-cpu-baseline > $OUT/c4_diag.log 2>&1 \
&& RAFTSTEP_DEBUG_WORK=1 timeout -k 10 200 python3 -u bench.py --workload C4 --steps 32 --warmup 16 --repeats 1 --no-cpu-baseline > $OUT/c4_work.log 2>&1
