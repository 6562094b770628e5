#!/bin/bash
# GPU session: full parity suite, then the C2 and C4 bench lines and a kernel-trace profile of C4.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
&& timeout -k 10 240 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench.log 2>&1 \
&& timeout -k 10 300 python -u bench.py --workload C4 --steps 100 --warmup 16 > $OUT/bench_c4.log 2>&1 \
&& timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_c4 -o run --output-format csv -- python -u bench.py --workload C4 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/prof_c4.log 2>&1
