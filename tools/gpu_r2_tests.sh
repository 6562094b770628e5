#!/bin/bash
# Round 2: the GPU test suite, then the bench lines (C2 headline with
# cpu_baseline, C3 on one GPU, C4), each step under its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r2t}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/gpu_tests.log 2>&1 || exit 1
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python -u bench.py > $OUT/bench_c2.log 2>&1 \
&& timeout -k 10 300 python -u bench.py --workload C3 --no-cpu-baseline > $OUT/bench_c3.log 2>&1 \
&& timeout -k 10 300 python -u bench.py --workload C4 --steps 64 --warmup 16 --no-cpu-baseline > $OUT/bench_c4.log 2>&1
