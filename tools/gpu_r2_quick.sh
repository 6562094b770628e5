#!/bin/bash
# GPU tests, then C2 / C3 / C4 bench lines (+ C4 with the one-pass kernel);
# NOTESTS=1 skips the tests.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2q}
mkdir -p $OUT
B="python3 -u bench.py --no-cpu-baseline"
step() { echo "== $(date +%T) $1" >> $OUT/progress.log; }
if [ -z "$NOTESTS" ]; then
step tests && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
fi
step c2 && timeout -k 10 200 $B > $OUT/bench_c2.log 2>&1 \
&& step c3 && timeout -k 10 200 $B --workload C3 > $OUT/bench_c3.log 2>&1 \
&& step c4 && timeout -k 10 200 $B --workload C4 --steps 64 --warmup 16 > $OUT/bench_c4.log 2>&1 \
&& step c4s && RAFTSTEP_TWO_PASS=0 timeout -k 10 200 $B --workload C4 --steps 64 --warmup 16 > $OUT/bench_c4_single.log 2>&1 \
&& step c5 && timeout -k 10 200 $B --workload C5 --steps 30 --warmup 5 > $OUT/bench_c5.log 2>&1 \
&& step done
