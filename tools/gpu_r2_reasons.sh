#!/bin/bash
# C4 deferral reasons (diaglib/: k_fast built with -DRAFTSTEP_DIAG_REASONS,
# loaded through RAFTSTEP_LIB) and the general kernel's worklist per window.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2reasons}
mkdir -p $OUT
B="python3 -u bench.py --no-cpu-baseline --workload C4 --steps 32 --warmup 200 --repeats 1"
RAFTSTEP_LIB=diaglib/libraftstep_diag.so RAFTSTEP_DEBUG_FAST=1 timeout -k 10 200 $B > $OUT/c4_reasons.log 2>&1 \
&& RAFTSTEP_DEBUG_WORK=1 timeout -k 10 200 $B > $OUT/c4_work.log 2>&1
