#!/bin/bash
# The whole GPU suite, then the bench lines at the driver's protocol
# (--steps 20 --warmup 5): C2 (with the CPU baseline, as the driver runs it),
# C4, C2 at 2^22 groups, C5, C3's one-GPU shard. Each step under its own limit.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r3full}
mkdir -p $OUT
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || exit 1
fi
B="python -u bench.py --steps 20 --warmup 5"
timeout -k 10 300 $B > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
timeout -k 10 300 $B --workload C4 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 1
timeout -k 10 300 $B --workload C2 --groups-per-gpu 4194304 --no-cpu-baseline > $OUT/bench_c2_4m.json 2> $OUT/bench_c2_4m.err || exit 1
timeout -k 10 300 $B --workload C5 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 1
timeout -k 10 300 $B --workload C3 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 1
