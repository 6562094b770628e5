#!/bin/bash
# Interleaved A/B of the working tree's library against diaglib/libraftstep_prev.so
# (the previous commit's k_fast) on C4, then the GPU tests of the working tree.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2abprev}
mkdir -p $OUT
B="python3 -u bench.py --no-cpu-baseline --workload C4 --steps 64 --warmup 200 --repeats 3"
step() { echo "== $(date +%T) $1" >> $OUT/progress.log; }
step ab && timeout -k 10 200 $B > $OUT/new_a.log 2>&1 \
&& RAFTSTEP_LIB=diaglib/libraftstep_prev.so timeout -k 10 200 $B > $OUT/prev_a.log 2>&1 \
&& timeout -k 10 200 $B > $OUT/new_b.log 2>&1 \
&& RAFTSTEP_LIB=diaglib/libraftstep_prev.so timeout -k 10 200 $B > $OUT/prev_b.log 2>&1 \
&& step tests && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
&& step done
