#!/bin/bash
# GPU tests, then C4 with one-wave list blocks and four-wave blocks
# (RAFTSTEP_LIST_BLOCK=64 / 256), interleaved, and C2.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2lb}
mkdir -p $OUT
B="python3 -u bench.py --no-cpu-baseline --workload C4 --steps 64 --warmup 200 --repeats 3"
step() { echo "== $(date +%T) $1" >> $OUT/progress.log; }
step tests && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
&& step ab && RAFTSTEP_LIST_BLOCK=64 timeout -k 10 200 $B > $OUT/c4_64a.log 2>&1 \
&& RAFTSTEP_LIST_BLOCK=256 timeout -k 10 200 $B > $OUT/c4_256a.log 2>&1 \
&& RAFTSTEP_LIST_BLOCK=64 timeout -k 10 200 $B > $OUT/c4_64b.log 2>&1 \
&& RAFTSTEP_LIST_BLOCK=256 timeout -k 10 200 $B > $OUT/c4_256b.log 2>&1 \
&& step c2 && timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > $OUT/c2.log 2>&1 \
&& step done
