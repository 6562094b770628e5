#!/bin/bash
# C4 diagnostics: general-kernel worklist size per launch and fast-kernel lane
# classes (both synchronising, so not a timing run), then a plain C4 bench line.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
RAFTSTEP_DEBUG_WORK=1 timeout -k 10 200 python3 -u bench.py --workload C4 --steps 64 --warmup 16 --no-cpu-baseline > $OUT/c4_work.log 2>&1 \
&& RAFTSTEP_DEBUG_FAST=1 timeout -k 10 200 python3 -u bench.py --workload C4 --steps 64 --warmup 16 --no-cpu-baseline > $OUT/c4_fast.log 2>&1 \
&& timeout -k 10 200 python3 -u bench.py --workload C4 --steps 100 --warmup 16 --no-cpu-baseline > $OUT/c4_bench.log 2>&1
