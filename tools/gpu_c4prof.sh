#!/bin/bash
# C4 bench line + kernel-trace profile (RAFT tests first).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_raft.py -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests_raft.log 2>&1 \
&& timeout -k 10 300 python -u bench.py --workload C4 --steps 100 --warmup 16 > $OUT/bench_c4.log 2>&1 \
&& timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_c4 -o run --output-format csv -- python -u bench.py --workload C4 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/prof_c4.log 2>&1
